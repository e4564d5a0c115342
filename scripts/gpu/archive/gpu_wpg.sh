#!/bin/bash
# T3L: workers per workgroup (one per SIMD) x waves per CU
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=10000
timeout -k 10 500 python -u scripts/sweep_uts.py T3L HCLIB_HIP_WAVES_PER_CU=2,4 HCLIB_HIP_WPG=1,2,4 > gpurun_out/wpg_t3l.log 2>&1 && echo "t3l ok"
