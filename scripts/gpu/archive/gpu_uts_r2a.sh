#!/bin/bash
# round 2: full GPU parity, then the UTS occupancy sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=10000
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo "gpu tests ok" &&
timeout -k 10 300 python -u scripts/sweep_uts.py T1XL HCLIB_HIP_UTS_GEO_FIXED=0,1 HCLIB_HIP_WAVES_PER_CU=4,6,8 > gpurun_out/sweep_t1xl.log 2>&1 && echo "sweep ok" &&
timeout -k 10 200 python -u scripts/sweep_uts.py T1 HCLIB_HIP_WAVES_PER_CU=4,8 > gpurun_out/sweep_t1.log 2>&1 &&
timeout -k 10 200 python -u scripts/sweep_uts.py T3L HCLIB_HIP_WAVES_PER_CU=2 > gpurun_out/sweep_t3l.log 2>&1 && echo "all ok"
