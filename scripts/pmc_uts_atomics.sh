#!/bin/bash
# L2 atomics of the UTS search kernels (one counter per pass) + kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcua
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o t -- python3 scripts/uts_atomics_pmc_run.py > $OUT/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_ATOMIC_sum --output-format csv -d $OUT/atomic -o a -- python3 scripts/uts_atomics_pmc_run.py > $OUT/atomic.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_ATOMIC_sum --output-format csv -d $OUT/ea -o e -- python3 scripts/uts_atomics_pmc_run.py > $OUT/ea.log 2>&1 &&
echo pmc ok
