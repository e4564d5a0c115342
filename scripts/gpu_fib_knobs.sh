#!/bin/bash
# fib(30) knob sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=10000
timeout -k 10 300 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_WAVES_PER_CU=2,4,8 HCLIB_HIP_FIB_CHUNK=8,32 HCLIB_HIP_FIB_HUNGER=4,8,32 > gpurun_out/fib_knobs.log 2>&1 &&
timeout -k 10 200 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_CARRY=1,2 HCLIB_HIP_FIB_SPILL_LO=16,32,72 > gpurun_out/fib_knobs2.log 2>&1 && echo "all ok"
