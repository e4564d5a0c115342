#!/bin/bash
# round 4: full GPU suite + the bench line at HEAD
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r04/full_tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/r04/bench.json 2> gpurun_out/r04/bench.err &&
echo ok
