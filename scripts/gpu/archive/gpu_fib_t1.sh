#!/bin/bash
# fib defaults (chunk 32, 2 waves/CU): GPU tests; T1 chunk sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=10000
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo "tests ok" &&
timeout -k 10 100 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_CARRY=1,1 > gpurun_out/fib_default.log 2>&1 &&
timeout -k 10 200 python -u scripts/sweep_uts.py T1 HCLIB_HIP_CHUNK=16,32,64 HCLIB_HIP_HUNGER=8,32 > gpurun_out/t1_chunk.log 2>&1 && echo "all ok"
