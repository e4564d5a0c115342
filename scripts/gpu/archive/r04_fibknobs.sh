#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 300 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_FIB_SPILL_LO=16,32,64,128 HCLIB_HIP_FIB_SPILL_HI=256,512 HCLIB_HIP_FIB_HUNGER=8,32 > gpurun_out/r04/fibknobs_a.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_WAVES_PER_CU=1,2,3 HCLIB_HIP_FIB_CHUNK=16,32,64 HCLIB_HIP_DEQUES=64,256 > gpurun_out/r04/fibknobs_b.log 2>&1 &&
echo ok
