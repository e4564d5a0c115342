#!/bin/bash
# round 4: exit records + LDS finish scopes for fib
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_device_api.py tests/test_capi.py -m gpu -x -q --timeout 120 --timeout-method thread -k "uts or fib or cross_gpu or device or stats or kind" > gpurun_out/r04/fib_tests.log 2>&1 &&
timeout -k 10 200 python -u scripts/uts_probe.py T1 T1L T1XL:7 T1XL T3L fib30 > gpurun_out/r04/fib_probe.log 2>&1 &&
timeout -k 10 200 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_FIB_LOCAL=0,1 HCLIB_HIP_WAVES_PER_CU=2,4 > gpurun_out/r04/fib_sweep.log 2>&1 &&
timeout -k 10 240 env HCLIB_AMD_LIB=hclib_amd/lib/timeline/libhclib_amd.so python -u scripts/uts_timeline.py gpurun_out/r04/timeline_exit.jsonl T1 T1XL:7 > gpurun_out/r04/timeline_exit.log 2>&1 &&
echo ok
