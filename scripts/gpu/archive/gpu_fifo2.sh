#!/bin/bash
# FIFO batches + newest-first hunger spills (level-synchronous bias), T3L
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=10000
HCLIB_HIP_FIFO=1 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "uts and (T3 or t3)" > gpurun_out/fifo2_tests.log 2>&1 && echo "tests ok" &&
timeout -k 10 500 python -u scripts/sweep_uts.py T3L HCLIB_HIP_FIFO=0,1 HCLIB_HIP_SPILL_LO=65,72,96,128 > gpurun_out/fifo2_t3l.log 2>&1 && echo "t3l ok" &&
timeout -k 10 200 python -u scripts/sweep_uts.py T3L HCLIB_HIP_FIFO=1 HCLIB_HIP_WAVES_PER_CU=2,3 HCLIB_HIP_HUNGER=8,32 > gpurun_out/fifo2_t3l_b.log 2>&1 && echo "all ok"
