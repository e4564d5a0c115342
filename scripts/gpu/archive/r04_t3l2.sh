#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 500 python -u scripts/sweep_uts.py T3L HCLIB_HIP_WPG=1,2 HCLIB_HIP_WAVES_PER_CU=2,3,4 > gpurun_out/r04/t3l2_wpg.log 2>&1 &&
timeout -k 10 400 python -u scripts/sweep_uts.py T3L HCLIB_HIP_SPILL_LO=66,96,128 HCLIB_HIP_HUNGER=16,32,64 > gpurun_out/r04/t3l2_spill.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T3L HCLIB_HIP_CHUNK=32,64,128 HCLIB_HIP_SPILL_HI=256,512 > gpurun_out/r04/t3l2_chunk.log 2>&1 &&
echo ok
