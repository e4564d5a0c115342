#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 300 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_FIB_SEED=2,3 HCLIB_HIP_WAVES_PER_CU=3,4 HCLIB_HIP_FIB_SPILL_HI=192,256 > gpurun_out/r04/fibseed2_sweep.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_FIB_SEED=0,2 HCLIB_HIP_WAVES_PER_CU=2,3 >> gpurun_out/r04/fibseed2_sweep.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_FIB_SEED=2 HCLIB_HIP_WAVES_PER_CU=3 HCLIB_HIP_FIB_SPILL_LO=24,32,48 >> gpurun_out/r04/fibseed2_sweep.log 2>&1 &&
echo ok
