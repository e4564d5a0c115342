#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_device_api.py -m gpu -x -q --timeout 120 --timeout-method thread -k "uts or fib or finish" > gpurun_out/r04/carry_tests.log 2>&1 &&
timeout -k 10 400 python -u scripts/ab_libs_t3l.py T3L hclib_amd/lib/libhclib_amd.so hclib_amd/lib/carry_perm/libhclib_amd.so > gpurun_out/r04/carry_ab_t3l.log 2>&1 &&
timeout -k 10 300 python -u scripts/ab_libs_t3l.py T1XL hclib_amd/lib/libhclib_amd.so hclib_amd/lib/carry_perm/libhclib_amd.so > gpurun_out/r04/carry_ab_t1xl.log 2>&1 &&
timeout -k 10 200 python -u scripts/ab_libs_t3l.py T1 hclib_amd/lib/libhclib_amd.so hclib_amd/lib/carry_perm/libhclib_amd.so > gpurun_out/r04/carry_ab_t1.log 2>&1 &&
echo ok
