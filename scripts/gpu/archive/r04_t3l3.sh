#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 500 python -u scripts/sweep_uts.py T3L HCLIB_HIP_SPILL_LO=65,66,67,68,70,72 HCLIB_HIP_HUNGER=16,32 > gpurun_out/r04/t3l3_spill.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T3L HCLIB_HIP_SPILL_LO=66,72 HCLIB_HIP_HUNGER=16,32 >> gpurun_out/r04/t3l3_spill.log 2>&1 &&
echo ok
