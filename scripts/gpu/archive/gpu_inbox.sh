#!/bin/bash
# LDS sibling hand-off (WPG worker waves per workgroup) on BIN trees: parity + A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=10000
HCLIB_HIP_WPG=2 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "uts and not cross" > gpurun_out/inbox_tests.log 2>&1 && echo "tests ok" &&
timeout -k 10 400 python -u scripts/sweep_uts.py T3L HCLIB_HIP_WAVES_PER_CU=2 HCLIB_HIP_WPG=1,2,1,2 > gpurun_out/inbox_t3l.log 2>&1 &&
timeout -k 10 400 python -u scripts/sweep_uts.py T3L HCLIB_HIP_WAVES_PER_CU=4 HCLIB_HIP_WPG=2,4 > gpurun_out/inbox_t3l4.log 2>&1 && echo "all ok"
