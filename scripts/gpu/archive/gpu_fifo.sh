#!/bin/bash
# T3L / T1: FIFO (oldest-first) ring batches vs LIFO, x waves per CU and spill_lo (A/B, interleaved)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=10000
timeout -k 10 400 python -u scripts/sweep_uts.py T3L HCLIB_HIP_WAVES_PER_CU=2,4 HCLIB_HIP_SPILL_LO=72,96 HCLIB_HIP_FIFO=0,1 > gpurun_out/fifo_t3l.log 2>&1 && echo "t3l ok" &&
timeout -k 10 200 python -u scripts/sweep_uts.py T3L HCLIB_HIP_FIFO=0,1,0,1 > gpurun_out/fifo_t3l_ab.log 2>&1 && echo "ab ok" &&
timeout -k 10 200 python -u scripts/sweep_uts.py T1 HCLIB_HIP_FIFO=0,1 > gpurun_out/fifo_t1.log 2>&1 && echo "all ok"
timeout -k 10 120 python -u -c "
import os, torch, hclib_amd as H
H.init(0)
for f in ('0', '1'):
    os.environ['HCLIB_HIP_FIFO'] = f
    r = H.uts('-t 0 -b 2000 -q 0.200014 -m 5 -r 7')
    print('fifo', f, {k: r[k] for k in r if k != 'levels'}, flush=True)
" > gpurun_out/fifo_stats.log 2>&1 && echo "stats ok"
