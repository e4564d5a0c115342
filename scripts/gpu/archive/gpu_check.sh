#!/bin/bash
# One GPU-box pass: parity tests, bench line, rocprofv3 kernel stats.
# Every GPU step has its own time limit; steps chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export HCLIB_HIP_SPIN_LIMIT_MS=${HCLIB_HIP_SPIN_LIMIT_MS:-10000}
timeout -k 10 600 python -m pytest tests -x -q -m gpu --timeout 300 > gpurun_out/gpu_tests.log 2>&1 && echo "tests ok" &&
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && echo "bench ok" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err && echo "prof ok"
