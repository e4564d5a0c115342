#!/bin/bash
# fib(30) knob sweep around the chunk-32 / 2-waves optimum
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=10000
timeout -k 10 400 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_WAVES_PER_CU=1,2,3 HCLIB_HIP_FIB_CHUNK=32,48,64 HCLIB_HIP_FIB_HUNGER=6,8,12 > gpurun_out/fib_knobs3.log 2>&1 &&
timeout -k 10 200 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_WAVES_PER_CU=2 HCLIB_HIP_FIB_CHUNK=32,64 HCLIB_HIP_FIB_SPILL_LO=16,32,48 > gpurun_out/fib_knobs4.log 2>&1 && echo "all ok"
