#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 500 python -u scripts/sweep_uts.py T3L HCLIB_HIP_WPG=2,4 HCLIB_HIP_WAVES_PER_CU=2,4 > gpurun_out/r04/t3l_wpg2.log 2>&1 &&
timeout -k 10 500 python -u scripts/sweep_uts.py T3L HCLIB_HIP_WPG=4,2 HCLIB_HIP_WAVES_PER_CU=4,2 >> gpurun_out/r04/t3l_wpg2.log 2>&1 &&
echo ok
