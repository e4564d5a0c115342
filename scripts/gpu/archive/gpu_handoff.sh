#!/bin/bash
# chunk hand-off v2 (paired seq/cnt, fast tickets, deferred publish): GPU tests, then A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=10000
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo "tests ok" &&
timeout -k 10 300 python -u scripts/sweep_uts.py T3L HCLIB_HIP_DEFER=0,1,0,1 > gpurun_out/handoff_t3l.log 2>&1 && echo "t3l ok" &&
timeout -k 10 300 python -u scripts/sweep_uts.py T3L HCLIB_HIP_SPILL_LO=65,72,96 > gpurun_out/handoff_t3l_spill.log 2>&1 && echo "spill ok" &&
timeout -k 10 300 python -u scripts/sweep_uts.py T1XL HCLIB_HIP_DEFER=0,1 > gpurun_out/handoff_t1xl.log 2>&1 && echo "t1xl ok" &&
timeout -k 10 200 python -u scripts/sweep_uts.py T1 HCLIB_HIP_DEFER=0,1 > gpurun_out/handoff_t1.log 2>&1 && echo "t1 ok" &&
timeout -k 10 200 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_CARRY=1 > gpurun_out/handoff_fib.log 2>&1 && echo "all ok"
