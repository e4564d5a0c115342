#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
HCLIB_HIP_SW_PK=1 timeout -k 10 120 python -u scripts/sw_dag_trace.py gpurun_out/r04/tr_pk1.bin > gpurun_out/r04/sw_trace_pk1.json 2>&1 &&
HCLIB_HIP_SW_PK=2 timeout -k 10 120 python -u scripts/sw_dag_trace.py gpurun_out/r04/tr_pk2.bin > gpurun_out/r04/sw_trace_pk2.json 2>&1 &&
rm -f gpurun_out/r04/tr_pk*.bin &&
HCLIB_HIP_FIB_LOCAL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_device_api.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fib or finish" > gpurun_out/r04/fiblds_tests.log 2>&1 &&
HCLIB_HIP_FIB_DEBUG=1 HCLIB_HIP_FIB_LOCAL=1 timeout -k 10 60 python -u -c "import hclib_amd as H; H.init(0); print(H.fib(30)); print(H.fib(30))" > gpurun_out/r04/fiblds_dbg.log 2>&1 &&
timeout -k 10 400 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_FIB_LOCAL=0,1 HCLIB_HIP_WAVES_PER_CU=2,4 HCLIB_HIP_FIB_CHUNK=16,32 > gpurun_out/r04/fiblds_sweep.log 2>&1 &&
echo ok
