#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_device_api.py tests/test_capi.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fib or finish" > gpurun_out/r04/fibseed_tests.log 2>&1 &&
HCLIB_HIP_FIB_SEED=1 timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_device_api.py tests/test_capi.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fib" >> gpurun_out/r04/fibseed_tests.log 2>&1 &&
HCLIB_HIP_FIB_SEED=1 timeout -k 10 60 python -u -c "import hclib_amd as H; H.init(0); print([H.fib(n)[0] for n in range(0, 16)])" >> gpurun_out/r04/fibseed_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_FIB_SEED=0,1,2,4 HCLIB_HIP_WAVES_PER_CU=2,3 HCLIB_HIP_FIB_SPILL_HI=256,384 > gpurun_out/r04/fibseed_sweep.log 2>&1 &&
echo ok
