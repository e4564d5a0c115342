#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 300 env HCLIB_HIP_UTS_SEED=1 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "uts" > gpurun_out/r04/seed2_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T1 HCLIB_HIP_UTS_SEED=1 HCLIB_HIP_UTS_RING=256,512 HCLIB_HIP_WAVES_PER_CU=2,4,8 HCLIB_HIP_SEED_PER_WAVE=8,32 > gpurun_out/r04/seed2_t1.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T1 HCLIB_HIP_UTS_SEED=1 HCLIB_HIP_UTS_RING=512 HCLIB_HIP_WAVES_PER_CU=4 HCLIB_HIP_SPILL_LO_HUNGRY=0,72,136 HCLIB_HIP_SPREAD=0,2 > gpurun_out/r04/seed2_t1_tail.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T1XL:7 HCLIB_HIP_UTS_SEED=1 HCLIB_HIP_SEED_PER_WAVE=8,32 HCLIB_HIP_SPILL_LO_HUNGRY=0,136 > gpurun_out/r04/seed2_t1xl7.log 2>&1 &&
timeout -k 10 200 env HCLIB_AMD_LIB=hclib_amd/lib/timeline/libhclib_amd.so HCLIB_HIP_UTS_SEED=1 HCLIB_HIP_UTS_RING=512 HCLIB_HIP_WAVES_PER_CU=4 python -u scripts/uts_timeline.py gpurun_out/r04/timeline_t1_seed2.jsonl T1 T1XL:7 > gpurun_out/r04/timeline_t1_seed2.log 2>&1 &&
echo ok
