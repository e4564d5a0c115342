#!/bin/bash
# GEO trees: LDS tail search for numChildren; parity + throughput
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=10000
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "uts" > gpurun_out/geo_tests.log 2>&1 && echo "tests ok" &&
timeout -k 10 200 python -u scripts/probe_chunks.py > gpurun_out/probe_chunks.log 2>&1 && echo "probe ok" &&
timeout -k 10 400 python -u scripts/sweep_uts.py T1XL HCLIB_HIP_WAVES_PER_CU=4,8,10 > gpurun_out/geo_t1xl.log 2>&1 && echo "t1xl ok" &&
timeout -k 10 200 python -u scripts/sweep_uts.py T1 HCLIB_HIP_WAVES_PER_CU=2,4,8 HCLIB_HIP_UTS_RING=256,512 > gpurun_out/geo_t1.log 2>&1 && echo "all ok"
