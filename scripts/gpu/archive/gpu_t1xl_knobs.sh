#!/bin/bash
# T1XL knob sweep (spill_lo x hunger interval x chunk)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=10000
timeout -k 10 600 python -u scripts/sweep_uts.py T1XL HCLIB_HIP_SPILL_LO=64,96,160 HCLIB_HIP_HUNGER=8,32,128 > gpurun_out/t1xl_knobs.log 2>&1 && echo "ok1" &&
timeout -k 10 300 python -u scripts/sweep_uts.py T1XL HCLIB_HIP_CHUNK=16,32,64 HCLIB_HIP_SPILL_HI=384,512 > gpurun_out/t1xl_knobs2.log 2>&1 && echo "all ok"
