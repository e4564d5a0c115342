#!/bin/bash
# packed-half SW DAG: parity tests, same-box A/B against the band form, critical-path trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/pk}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "packed_half or generic_promise_dag or both_schedules or multiwave" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 200 python -u scripts/sw_pk_ab.py 3 > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
grep pk= $OUT/ab.log
timeout -k 10 120 python -u scripts/sw_dag_trace.py $OUT/trace.bin > $OUT/trace.json 2> $OUT/trace.err || { tail -5 $OUT/trace.err; exit 1; }
rm -f $OUT/trace.bin
python3 -c "
import json; d=json.load(open('$OUT/trace.json'))
print('plain', d['plain_ms'], 'traced', d['traced_ms'])
for k in ('row','col','all'):
    r=d[k]; print(k, {x: r[x] for x in ('release_us','pickup_us','body_us','put_us','in_ingress_us','in_wave0_us','in_wave1_us')})
"
