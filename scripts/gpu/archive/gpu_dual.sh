#!/bin/bash
# two-slot narrow loop (BIN trees): GPU tests + A/B on T3L / T3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=10000
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo "tests ok" &&
timeout -k 10 300 python -u scripts/sweep_uts.py T3L HCLIB_HIP_DUAL=0,1,0,1 > gpurun_out/dual_t3l.log 2>&1 &&
timeout -k 10 400 python -u scripts/sweep_uts.py T3L HCLIB_HIP_DUAL=1 HCLIB_HIP_SPILL_LO=72,96,136,160 > gpurun_out/dual_t3l_spill.log 2>&1 && echo "all ok"
