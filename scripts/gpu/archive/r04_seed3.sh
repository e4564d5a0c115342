#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000 HCLIB_HIP_UTS_SEED=1
timeout -k 10 300 python -u scripts/sweep_uts.py T1 HCLIB_HIP_UTS_RING=512 HCLIB_HIP_WAVES_PER_CU=4 HCLIB_HIP_SEED_PER_WAVE=2,4,8 HCLIB_HIP_SPILL_LO=96,160,224 > gpurun_out/r04/seed3_t1.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T1L HCLIB_HIP_WAVES_PER_CU=4,8 HCLIB_HIP_SEED_PER_WAVE=4,8,32 HCLIB_HIP_SPILL_LO=160,224 > gpurun_out/r04/seed3_t1l.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T1XL:7 HCLIB_HIP_SEED_PER_WAVE=8,32 HCLIB_HIP_SPILL_LO=160,224,336 > gpurun_out/r04/seed3_t1xl7.log 2>&1 &&
timeout -k 10 200 env HCLIB_AMD_LIB=hclib_amd/lib/timeline/libhclib_amd.so HCLIB_HIP_SEED_PER_WAVE=32 python -u scripts/uts_timeline.py gpurun_out/r04/timeline_t1xl7_seed3.jsonl T1XL:7 > gpurun_out/r04/timeline_t1xl7_seed3.log 2>&1 &&
echo ok
