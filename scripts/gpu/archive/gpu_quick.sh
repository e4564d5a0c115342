#!/bin/bash
# quick check of the current tree: GPU tests, T3L / T1XL / T1 / fib times
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=10000
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo "tests ok" &&
timeout -k 10 200 python -u scripts/sweep_uts.py T3L HCLIB_HIP_CARRY=2,2 > gpurun_out/quick_t3l.log 2>&1 &&
timeout -k 10 200 python -u scripts/sweep_uts.py T1XL HCLIB_HIP_CARRY=2 > gpurun_out/quick_t1xl.log 2>&1 &&
timeout -k 10 100 python -u scripts/sweep_uts.py T1 HCLIB_HIP_CARRY=2 > gpurun_out/quick_t1.log 2>&1 &&
timeout -k 10 100 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_CARRY=1 > gpurun_out/quick_fib.log 2>&1 && echo "all ok"
