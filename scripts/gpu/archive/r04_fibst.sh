#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
HCLIB_AMD_LIB=hclib_amd/lib/stamps/libhclib_amd.so timeout -k 10 120 python -u scripts/fib_stamps.py > gpurun_out/r04/fib_stamps2.log 2>&1 && echo ok
