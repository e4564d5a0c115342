#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_device_api.py tests/test_capi.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fib or finish" > gpurun_out/r04/seedbulk_tests.log 2>&1 &&
timeout -k 10 60 python -u -c "import hclib_amd as H; H.init(0); print([H.fib(n)[0] for n in range(0, 16)])" >> gpurun_out/r04/seedbulk_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/ab_libs_fib.py 30 hclib_amd/lib/libhclib_amd.so hclib_amd/lib/base/libhclib_amd.so > gpurun_out/r04/seedbulk_ab.log 2>&1 &&
timeout -k 10 300 python -u scripts/ab_libs_fib.py 30 hclib_amd/lib/libhclib_amd.so hclib_amd/lib/base/libhclib_amd.so >> gpurun_out/r04/seedbulk_ab.log 2>&1 &&
echo ok
