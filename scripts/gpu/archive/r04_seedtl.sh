#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000 HCLIB_HIP_UTS_SEED=1
timeout -k 10 200 env HCLIB_AMD_LIB=hclib_amd/lib/timeline/libhclib_amd.so HCLIB_HIP_UTS_RING=512 HCLIB_HIP_WAVES_PER_CU=4 python -u scripts/uts_timeline.py gpurun_out/r04/timeline_seedlv_t1.jsonl T1 > gpurun_out/r04/timeline_seedlv.log 2>&1 &&
timeout -k 10 200 env HCLIB_AMD_LIB=hclib_amd/lib/timeline/libhclib_amd.so HCLIB_HIP_SEED_PER_WAVE=32 python -u scripts/uts_timeline.py gpurun_out/r04/timeline_seedlv_t1xl7.jsonl T1XL:7 >> gpurun_out/r04/timeline_seedlv.log 2>&1 &&
echo ok
