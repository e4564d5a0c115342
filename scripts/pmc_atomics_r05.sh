#!/bin/bash
# Round 5: counted L2 atomics (TCC_ATOMIC_sum, TCC_EA0_ATOMIC_sum: one counter
# per pass) of fib(30), UTS T1 and T1XL at HEAD, plus the kernel-trace pass
# of the same workload; reduce with scripts/atomics_pmc_summary.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcat
rm -rf $OUT; mkdir -p $OUT
HCLIB_HIP_FIB_DEBUG=1 timeout -k 10 120 python3 scripts/atomics_pmc_r05.py > $OUT/plain.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o t -- python3 scripts/atomics_pmc_r05.py > $OUT/trace.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc TCC_ATOMIC_sum --output-format csv -d $OUT/atomic -o a -- python3 scripts/atomics_pmc_r05.py > $OUT/atomic.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_ATOMIC_sum --output-format csv -d $OUT/ea -o e -- python3 scripts/atomics_pmc_r05.py > $OUT/ea.log 2>&1 &&
echo pmc ok
