#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
HCLIB_AMD_LIB=hclib_amd/lib/fib_small/libhclib_amd.so timeout -k 10 100 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fib30" > gpurun_out/r04/fibsmall_tests.log 2>&1 &&
HCLIB_AMD_LIB=hclib_amd/lib/fib_small/libhclib_amd.so timeout -k 10 300 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_WAVES_PER_CU=2,4,6,8 HCLIB_HIP_FIB_SPILL_HI=128,256 > gpurun_out/r04/fibsmall_sweep.log 2>&1 &&
timeout -k 10 200 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_WAVES_PER_CU=2,3 > gpurun_out/r04/fibsmall_base.log 2>&1 &&
echo ok
