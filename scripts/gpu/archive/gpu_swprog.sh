#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 240 python -u -m pytest tests/test_gpu.py -x -v -m gpu -k "sw" --timeout 120 --timeout-method thread > gpurun_out/swprog_tests.log 2>&1 && echo "sw tests ok" &&
timeout -k 10 120 python -u scripts/sw_progressive_ab.py > gpurun_out/sw_progressive_ab.log 2>&1 && echo "ab ok" && cat gpurun_out/sw_progressive_ab.log
