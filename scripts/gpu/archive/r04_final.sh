#!/bin/bash
# round 4: full GPU suite, the bench line, and the rocprof kernel summary of the same command
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r04/full_tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/r04/bench.json 2> gpurun_out/r04/bench.err &&
rm -rf gpurun_out/r04/prof &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r04/prof -o run -- python3 -u bench.py > gpurun_out/r04/bench_prof.json 2> gpurun_out/r04/bench_prof.err &&
echo ok
