#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 500 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_FIB_HUNGER=8,16,32 HCLIB_HIP_FIB_SPILL_LO=32,64 HCLIB_HIP_FIB_SPILL_HI=256,320 > gpurun_out/r04/fibknobs_g.log 2>&1 &&
echo ok
