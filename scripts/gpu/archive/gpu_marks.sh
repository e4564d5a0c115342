#!/bin/bash
# push_outputs: tagged-mark lane-per-output form vs per-lane piece loop
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=10000
timeout -k 10 400 python -u scripts/sweep_uts.py T1XL HCLIB_HIP_MARKS=1,0,1,0 > gpurun_out/marks_t1xl.log 2>&1 && echo "t1xl ok" &&
timeout -k 10 200 python -u scripts/sweep_uts.py T1 HCLIB_HIP_MARKS=1,0,1,0 > gpurun_out/marks_t1.log 2>&1 && echo "t1 ok" &&
timeout -k 10 200 python -u scripts/sweep_uts.py T3L HCLIB_HIP_MARKS=1,0 > gpurun_out/marks_t3l.log 2>&1 && echo "all ok"
