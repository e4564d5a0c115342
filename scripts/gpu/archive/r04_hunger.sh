#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000 HCLIB_HIP_SPREAD=2
timeout -k 10 300 python -u scripts/sweep_uts.py T1 HCLIB_HIP_UTS_RING=512 HCLIB_HIP_WAVES_PER_CU=4,8 HCLIB_HIP_HUNGER_FAST=1,2,4,16 HCLIB_HIP_HUNGER=16,64 > gpurun_out/r04/hunger_t1.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T1XL:7 HCLIB_HIP_HUNGER_FAST=1,2,4,16 > gpurun_out/r04/hunger_t1xl7.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T1XL HCLIB_HIP_HUNGER_FAST=1,4,16 > gpurun_out/r04/hunger_t1xl.log 2>&1 &&
echo ok
