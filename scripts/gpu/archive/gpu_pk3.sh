#!/bin/bash
# packed-half SW DAG: parity, variant A/B (HEAD single-wave build in lib/pk1w), trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/pk}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "packed_half or generic_promise_dag or both_schedules or dag or sw" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u scripts/sw_pk_variants.py hclib_amd/lib/libhclib_amd.so $VARIANTS > $OUT/variants.log 2>&1 || { tail -5 $OUT/variants.log; exit 1; }
cat $OUT/variants.log
timeout -k 10 120 python -u scripts/sw_dag_trace.py $OUT/trace.bin > $OUT/trace.json 2> $OUT/trace.err || { tail -5 $OUT/trace.err; exit 1; }
rm -f $OUT/trace.bin
python3 -c "
import json; d=json.load(open('$OUT/trace.json'))
print('plain', d['plain_ms'], 'traced', d['traced_ms'])
for k in ('row','col','all'):
    r=d[k]; print(k, {x: r[x] for x in ('release_us','pickup_us','body_us','put_us','in_ingress_us','in_w0_loop_us','in_wave0_us','in_wave1_us')})
"
