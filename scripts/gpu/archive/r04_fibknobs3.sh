#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 400 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_FIB_HUNGER=4,8,16 HCLIB_HIP_FIB_CHUNK=16,32,64 > gpurun_out/r04/fibknobs_e.log 2>&1 &&
timeout -k 10 400 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_FIB_SPILL_LO=32,64 HCLIB_HIP_FIB_SPILL_HI=256,320 HCLIB_HIP_FIB_CLIMB=1073741824,0 > gpurun_out/r04/fibknobs_f.log 2>&1 &&
echo ok
