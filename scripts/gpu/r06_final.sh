#!/bin/bash
# round 6 final: full GPU suite, smoke, the bench line + its rocprof kernel
# summary, then the PMC passes (triad HBM bytes; UTS SQ counters on T1XL and
# T3L; counted L2 atomics of fib(30), T1 and T1XL) and the triad mix ceiling
# (FULL=0: suite, smoke and bench only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/full_tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")" > $OUT/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err &&
if [ "${FULL:-1}" = 0 ]; then echo ok; exit 0; fi &&
rm -rf $OUT/prof &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u bench.py > $OUT/bench_prof.json 2> $OUT/bench_prof.err &&
rm -rf gpurun_out/pmc gpurun_out/pmcu_t1xl gpurun_out/pmcu_t3l &&
bash scripts/pmc_triad.sh > $OUT/pmc_triad.log 2>&1 &&
bash scripts/pmc_uts.sh T1XL 0 gpurun_out/pmcu_t1xl > $OUT/pmc_t1xl.log 2>&1 &&
bash scripts/pmc_uts.sh T3L 0 gpurun_out/pmcu_t3l > $OUT/pmc_t3l.log 2>&1 &&
bash scripts/pmc_atomics_r05.sh > $OUT/pmc_atomics.log 2>&1 &&
timeout -k 10 200 scripts/ubench/ub_triad_ceiling.bin > $OUT/triad_ceiling.jsonl 2>&1 &&
echo ok
