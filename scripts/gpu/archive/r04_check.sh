#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "uts or fib" > gpurun_out/r04/check_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T3L HCLIB_HIP_WPG=2 > gpurun_out/r04/check_t3l.log 2>&1 &&
echo ok
