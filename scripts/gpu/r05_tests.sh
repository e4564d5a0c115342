#!/bin/bash
# round 5: the GPU suite (optionally a -k filter) and, with BENCH=1, one bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r05; mkdir -p $OUT
export TMPDIR=/tmp
TAG=${TAG:-tests}
if [ -n "$K" ]; then KF=(-k "$K"); else KF=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${KF[@]}" > $OUT/$TAG.log 2>&1
rc=$?
tail -3 $OUT/$TAG.log
[ $rc -ne 0 ] && exit $rc
if [ "$BENCH" = 1 ]; then
  timeout -k 10 400 python -u bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench_$TAG.json'))
c=d['configs']
print('T3L kernel ms', round(d['config']['uts_kernel_ms_rank0'],3), 'T1', round(c['uts_t1_1gpu']['kernel_ms'],4), 'fib30', round(c['fib30_gpu']['kernel_ms'],4), 'sw rows', round(c['sw_64k']['kernel_ms'],3), 'sw dag', round(c['sw_64k_promise_dag']['kernel_ms'],3), 'T1XL', round(d['wide_tree']['kernel_ms_per_rank'][0],2), 'triad frac', round(d['roofline']['frac'],3))
"
fi
