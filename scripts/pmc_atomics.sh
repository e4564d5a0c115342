#!/bin/bash
# L2 atomic counters of the calibration kernels and of the fib megakernel,
# one counter per pass, plus the kernel-trace stats of the same workload.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmca
mkdir -p $OUT
timeout -k 10 120 python3 scripts/atomics_pmc_run.py > $OUT/plain.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o t -- python3 scripts/atomics_pmc_run.py > $OUT/trace.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc TCC_ATOMIC_sum --output-format csv -d $OUT/atomic -o a -- python3 scripts/atomics_pmc_run.py > $OUT/atomic.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_ATOMIC_sum --output-format csv -d $OUT/ea -o e -- python3 scripts/atomics_pmc_run.py > $OUT/ea.log 2>&1 &&
echo pmc ok
