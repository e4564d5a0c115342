#!/bin/bash
# round 2: UTS parity, T3L tight narrow loop A/B, GEO ring size x waves/CU sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=10000
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "uts or fib" > gpurun_out/uts_tests.log 2>&1 && echo "uts tests ok" &&
timeout -k 10 300 python -u scripts/sweep_uts.py T3L HCLIB_HIP_CARRY=1,2,1,2 > gpurun_out/t3l_carry_ab.log 2>&1 && echo "t3l ok" &&
timeout -k 10 400 python -u scripts/sweep_uts.py T1XL HCLIB_HIP_UTS_RING=256,512 HCLIB_HIP_WAVES_PER_CU=8,10,12 > gpurun_out/sweep_ring.log 2>&1 && echo "sweep ok" &&
timeout -k 10 200 python -u scripts/sweep_uts.py T1 HCLIB_HIP_UTS_RING=256,512 HCLIB_HIP_WAVES_PER_CU=4,8 > gpurun_out/sweep_ring_t1.log 2>&1 && echo "all ok"
