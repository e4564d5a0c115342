#!/bin/bash
# round 6: the GPU suite (optionally a -k filter K), then optional steps:
# SHARD=1 the T3L 8-shard A/B of hclib_amd/lib/base_r05 against HEAD's
# library; BENCH=1 one bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06; mkdir -p $OUT
export TMPDIR=/tmp
TAG=${TAG:-tests}
if [ -n "$K" ]; then KF=(-k "$K"); else KF=(); fi
if [ "$SKIPTESTS" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${KF[@]}" > $OUT/$TAG.log 2>&1
  rc=$?
  tail -3 $OUT/$TAG.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ "$SHARD" = 1 ]; then
  for rep in 1 2; do
    TREE=T3L timeout -k 10 300 python -u scripts/shard_ab.py 3 base=hclib_amd/lib/base_r05/libhclib_amd.so new=hclib_amd/lib/libhclib_amd.so >> $OUT/shard_t3l_$TAG.log 2>&1 || exit $?
  done
  cat $OUT/shard_t3l_$TAG.log
fi
if [ "$BENCH" = 1 ]; then
  timeout -k 10 400 python -u bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/bench_$TAG.json'))
c=d['configs']
print('T3L kernel ms', round(d['config']['uts_kernel_ms_rank0'],3), 'T1', round(c['uts_t1_1gpu']['kernel_ms'],4), 'fib30', round(c['fib30_gpu']['kernel_ms'],4), 'sw rows', round(c['sw_64k']['kernel_ms'],3), 'sw dag', round(c['sw_64k_promise_dag']['kernel_ms'],3), 'T1XL', round(d['wide_tree']['kernel_ms_per_rank'][0],2), 'triad frac', round(d['roofline']['frac'],3))
"
fi
echo done
