#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
rm -f gpurun_out/r04/fib_tl2.jsonl
HCLIB_AMD_LIB=hclib_amd/lib/timeline/libhclib_amd.so timeout -k 10 120 python -u scripts/uts_timeline.py gpurun_out/r04/fib_tl2.jsonl fib30 > gpurun_out/r04/fib_tl2.log 2>&1 &&
echo ok
