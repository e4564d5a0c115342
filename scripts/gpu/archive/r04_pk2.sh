#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "packed" > gpurun_out/r04/pk2_tests.log 2>&1 &&
timeout -k 10 200 python -u scripts/sw_pk_ab.py 5 1 2 > gpurun_out/r04/pk2_ab.log 2>&1 &&
echo ok
