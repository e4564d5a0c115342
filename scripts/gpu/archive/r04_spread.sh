#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 300 python -u scripts/sweep_uts.py T1 HCLIB_HIP_UTS_RING=256,512 HCLIB_HIP_WAVES_PER_CU=2,4,8 HCLIB_HIP_SPREAD=0,1,2 > gpurun_out/r04/spread_t1.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T1XL:7 HCLIB_HIP_SPREAD=0,1,2 > gpurun_out/r04/spread_t1xl7.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T3L HCLIB_HIP_SPREAD=0,1,2 > gpurun_out/r04/spread_t3l.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T1XL HCLIB_HIP_SPREAD=0,1,2 > gpurun_out/r04/spread_t1xl.log 2>&1 &&
timeout -k 10 200 env HCLIB_AMD_LIB=hclib_amd/lib/timeline/libhclib_amd.so HCLIB_HIP_UTS_RING=512 HCLIB_HIP_WAVES_PER_CU=8 HCLIB_HIP_SPREAD=2 python -u scripts/uts_timeline.py gpurun_out/r04/timeline_t1_spread2.jsonl T1 > gpurun_out/r04/timeline_t1_spread2.log 2>&1 &&
echo ok
