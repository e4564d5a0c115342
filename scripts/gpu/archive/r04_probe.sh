#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 200 env HCLIB_AMD_LIB=hclib_amd/lib/timeline/libhclib_amd.so HCLIB_HIP_UTS_RING=512 HCLIB_HIP_WAVES_PER_CU=8 HCLIB_HIP_SPREAD=2 python -u scripts/uts_timeline.py gpurun_out/r04/timeline_t1_probe.jsonl T1 > gpurun_out/r04/timeline_t1_probe.log 2>&1 &&
echo ok
