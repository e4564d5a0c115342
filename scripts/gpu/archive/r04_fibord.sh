#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_device_api.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fib or finish" > gpurun_out/r04/fibord_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/ab_libs_fib.py 30 hclib_amd/lib/libhclib_amd.so hclib_amd/lib/fib_base/libhclib_amd.so > gpurun_out/r04/fibord_ab.log 2>&1 &&
HCLIB_AMD_LIB=hclib_amd/lib/stamps/libhclib_amd.so timeout -k 10 120 python -u scripts/fib_stamps.py > gpurun_out/r04/fib_stamps8.log 2>&1 &&
echo ok
