#!/bin/bash
# T3L knob sweep on the current tree (waves per CU x spill_lo x hunger interval)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=10000
timeout -k 10 500 python -u scripts/sweep_uts.py T3L HCLIB_HIP_WAVES_PER_CU=2,3,4 HCLIB_HIP_SPILL_LO=65,72 HCLIB_HIP_HUNGER=8,32 > gpurun_out/sweep_t3l.log 2>&1 && echo "t3l ok" &&
timeout -k 10 300 python -u scripts/sweep_uts.py T3L HCLIB_HIP_BACKOFF=1,4,16 HCLIB_HIP_CHUNK=32,64 > gpurun_out/sweep_t3l_b.log 2>&1 && echo "all ok"
