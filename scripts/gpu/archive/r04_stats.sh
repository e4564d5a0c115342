#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "uts" > gpurun_out/r04/stats_tests.log 2>&1 &&
timeout -k 10 400 python -u scripts/ab_libs_t3l.py T3L hclib_amd/lib/libhclib_amd.so hclib_amd/lib/base/libhclib_amd.so > gpurun_out/r04/stats_ab_t3l.log 2>&1 &&
timeout -k 10 400 python -u scripts/ab_libs_t3l.py T3L hclib_amd/lib/libhclib_amd.so hclib_amd/lib/base/libhclib_amd.so >> gpurun_out/r04/stats_ab_t3l.log 2>&1 &&
echo ok
