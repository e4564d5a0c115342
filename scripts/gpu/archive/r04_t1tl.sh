#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 200 env HCLIB_AMD_LIB=hclib_amd/lib/timeline/libhclib_amd.so HCLIB_HIP_UTS_RING=512 HCLIB_HIP_WAVES_PER_CU=8 python -u scripts/uts_timeline.py gpurun_out/r04/timeline_t1_8wpc_q.jsonl T1 > gpurun_out/r04/timeline_t1_8wpc_q.log 2>&1 &&
timeout -k 10 200 env HCLIB_AMD_LIB=hclib_amd/lib/timeline/libhclib_amd.so python -u scripts/uts_timeline.py gpurun_out/r04/timeline_t1xl7_q.jsonl T1XL:7 > gpurun_out/r04/timeline_t1xl7_q.log 2>&1 &&
echo ok
timeout -k 10 300 python -u scripts/sweep_uts.py T1 HCLIB_HIP_UTS_RING=512 HCLIB_HIP_WAVES_PER_CU=8 HCLIB_HIP_RAMP_CHUNK=0,4,8,16 HCLIB_HIP_SPILL_LO_HUNGRY=0,136 > gpurun_out/r04/ramp_t1.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T1XL:7 HCLIB_HIP_RAMP_CHUNK=0,4,8,16 > gpurun_out/r04/ramp_t1xl7.log 2>&1 &&
echo ok2
