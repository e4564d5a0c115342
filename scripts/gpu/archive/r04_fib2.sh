#!/bin/bash
# round 4: fib LDS scopes diagnosis
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 100 env HCLIB_HIP_FIB_DEBUG=1 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_FIB_LOCAL=0,1 > gpurun_out/r04/fib_dbg.log 2>&1 &&
timeout -k 10 200 env HCLIB_AMD_LIB=hclib_amd/lib/timeline/libhclib_amd.so HCLIB_HIP_FIB_LOCAL=0 python -u scripts/uts_timeline.py gpurun_out/r04/timeline_fib_hbm.jsonl fib30 > gpurun_out/r04/timeline_fib.log 2>&1 &&
timeout -k 10 200 env HCLIB_AMD_LIB=hclib_amd/lib/timeline/libhclib_amd.so HCLIB_HIP_FIB_LOCAL=1 python -u scripts/uts_timeline.py gpurun_out/r04/timeline_fib_lds.jsonl fib30 >> gpurun_out/r04/timeline_fib.log 2>&1 &&
timeout -k 10 200 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_FIB_LOCAL=1 HCLIB_HIP_FIB_SPILL_LO=32,64,128 HCLIB_HIP_FIB_HUNGER=8,32 > gpurun_out/r04/fib_knobs.log 2>&1 &&
echo ok
