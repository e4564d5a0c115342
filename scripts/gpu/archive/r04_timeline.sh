#!/bin/bash
# round 4: UTS worker timelines (T1, T1L, T1XL 8-way shards) + T1 knob sweep on the product build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 240 env HCLIB_AMD_LIB=hclib_amd/lib/timeline/libhclib_amd.so python -u scripts/uts_timeline.py gpurun_out/r04/timeline.jsonl T1 T1L T1XL:7 > gpurun_out/r04/timeline.log 2>&1 &&
timeout -k 10 200 python -u scripts/sweep_uts.py T1 HCLIB_HIP_WAVES_PER_CU=2,4 HCLIB_HIP_SPILL_LO=16,32,64,128 > gpurun_out/r04/t1_sweep.log 2>&1 &&
timeout -k 10 200 python -u scripts/sweep_uts.py T1L HCLIB_HIP_SPILL_LO=64,128,224 > gpurun_out/r04/t1l_sweep.log 2>&1 &&
echo ok
