#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 100 env HCLIB_AMD_LIB=hclib_amd/lib/stamps/libhclib_amd.so python -u scripts/fib_stamps.py > gpurun_out/r04/fib_stamps.log 2>&1 &&
echo ok
