#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 500 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_FIB_SPILL_LO_HUNGRY=0,16,32 HCLIB_HIP_FIB_HUNGER_FAST=0,1 HCLIB_HIP_FIB_RAMP_CHUNK=0,16 > gpurun_out/r04/fibtail.log 2>&1 &&
echo ok
