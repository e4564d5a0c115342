#!/bin/bash
# narrow-loop hand-off of outputs beyond one batch to an idle sibling (WPG 2): parity + A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=10000
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "uts and not cross" > gpurun_out/inbox2_tests.log 2>&1 && echo "tests ok" &&
timeout -k 10 400 python -u scripts/sweep_uts.py T3L HCLIB_HIP_NARROW_HANDOFF=0,1,0,1 > gpurun_out/inbox2_t3l.log 2>&1 &&
timeout -k 10 400 python -u scripts/sweep_uts.py T3L HCLIB_HIP_NARROW_HANDOFF=1 HCLIB_HIP_SPILL_LO=72,96,128 > gpurun_out/inbox2_t3l_spill.log 2>&1 && echo "all ok"
