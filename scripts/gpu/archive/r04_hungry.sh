#!/bin/bash
# round 4: spill threshold while many waves are hungry (ramp-up / tail)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 200 python -u scripts/sweep_uts.py T1 HCLIB_HIP_SPILL_LO_HUNGRY=0,72,136 HCLIB_HIP_WAVES_PER_CU=2,4 > gpurun_out/r04/hungry_t1.log 2>&1 &&
timeout -k 10 200 python -u scripts/sweep_uts.py T1L HCLIB_HIP_SPILL_LO_HUNGRY=0,72,136 > gpurun_out/r04/hungry_t1l.log 2>&1 &&
timeout -k 10 200 python -u scripts/sweep_uts.py T1XL:7 HCLIB_HIP_SPILL_LO_HUNGRY=0,72,136 > gpurun_out/r04/hungry_t1xl7.log 2>&1 &&
timeout -k 10 200 python -u scripts/sweep_uts.py T1XL HCLIB_HIP_SPILL_LO_HUNGRY=0,136 > gpurun_out/r04/hungry_t1xl.log 2>&1 &&
echo ok
timeout -k 10 200 python -u scripts/sweep_uts.py T1 HCLIB_HIP_UTS_RING=512 HCLIB_HIP_WAVES_PER_CU=4,8 HCLIB_HIP_SPILL_LO_HUNGRY=0,136 > gpurun_out/r04/hungry_t1_512.log 2>&1 &&
timeout -k 10 240 env HCLIB_AMD_LIB=hclib_amd/lib/timeline/libhclib_amd.so python -u scripts/uts_timeline.py gpurun_out/r04/timeline_term2.jsonl T1 T1XL:7 > gpurun_out/r04/timeline_term2.log 2>&1 &&
echo ok2
