#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 400 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_FIB_SPILL_LO_HUNGRY=0,4,8,16 HCLIB_HIP_FIB_RAMP_CHUNK=0,8,16 > gpurun_out/r04/fibramp.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_FIB_HUNGER_FAST=0,1,2 HCLIB_HIP_FIB_HUNGER=4,8 > gpurun_out/r04/fibramp2.log 2>&1 &&
echo ok
