#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "uts or packed or sw_64k or fib or finish" > gpurun_out/r04/hoist_tests.log 2>&1 &&
timeout -k 10 400 python -u scripts/ab_libs_t3l.py T3L hclib_amd/lib/libhclib_amd.so hclib_amd/lib/nohoist/libhclib_amd.so > gpurun_out/r04/hoist_ab_t3l.log 2>&1 &&
timeout -k 10 400 python -u scripts/ab_libs_t3l.py T3L hclib_amd/lib/libhclib_amd.so hclib_amd/lib/nohoist/libhclib_amd.so >> gpurun_out/r04/hoist_ab_t3l.log 2>&1 &&
HCLIB_AMD_LIB=hclib_amd/lib/stamps/libhclib_amd.so timeout -k 10 120 python -u scripts/fib_stamps.py > gpurun_out/r04/fib_stamps7.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_FIB_CLIMB=1,2,3,4,8,1073741824 > gpurun_out/r04/fib_climbk.log 2>&1 &&
echo ok
