#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 500 python -u scripts/sweep_uts.py T3L HCLIB_HIP_UTS_DUAL=0,1 HCLIB_HIP_SPILL_LO=66,72,96 > gpurun_out/r04/t3l_dual.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T3L HCLIB_HIP_UTS_DUAL=1,0 > gpurun_out/r04/t3l_dual2.log 2>&1 &&
echo ok
