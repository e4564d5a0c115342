#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 300 env HCLIB_HIP_UTS_SEED=1 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "uts" > gpurun_out/r04/seed_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T1 HCLIB_HIP_UTS_SEED=0,1 HCLIB_HIP_UTS_RING=256,512 HCLIB_HIP_WAVES_PER_CU=2,4,8 > gpurun_out/r04/seed_t1.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T1XL:7 HCLIB_HIP_UTS_SEED=0,1 HCLIB_HIP_SEED_PER_WAVE=4,8,16 > gpurun_out/r04/seed_t1xl7.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T1L HCLIB_HIP_UTS_SEED=0,1 > gpurun_out/r04/seed_t1l.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T1XL HCLIB_HIP_UTS_SEED=0,1 > gpurun_out/r04/seed_t1xl.log 2>&1 &&
timeout -k 10 200 env HCLIB_AMD_LIB=hclib_amd/lib/timeline/libhclib_amd.so HCLIB_HIP_UTS_SEED=1 HCLIB_HIP_UTS_RING=512 HCLIB_HIP_WAVES_PER_CU=8 python -u scripts/uts_timeline.py gpurun_out/r04/timeline_t1_seed.jsonl T1 > gpurun_out/r04/timeline_t1_seed.log 2>&1 &&
echo ok
