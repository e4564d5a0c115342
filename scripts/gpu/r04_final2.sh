#!/bin/bash
# round 4 final: full GPU suite, the bench line + its rocprof kernel summary,
# then the PMC passes (triad HBM bytes; UTS SQ counters on T1XL and T3L)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r04/full_tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/r04/bench.json 2> gpurun_out/r04/bench.err &&
rm -rf gpurun_out/r04/prof &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r04/prof -o run -- python3 -u bench.py > gpurun_out/r04/bench_prof.json 2> gpurun_out/r04/bench_prof.err &&
rm -rf gpurun_out/pmc gpurun_out/pmcu_t1xl gpurun_out/pmcu_t3l &&
bash scripts/pmc_triad.sh > gpurun_out/r04/pmc_triad.log 2>&1 &&
bash scripts/pmc_uts.sh T1XL 0 gpurun_out/pmcu_t1xl > gpurun_out/r04/pmc_t1xl.log 2>&1 &&
bash scripts/pmc_uts.sh T3L 0 gpurun_out/pmcu_t3l > gpurun_out/r04/pmc_t3l.log 2>&1 &&
echo ok
