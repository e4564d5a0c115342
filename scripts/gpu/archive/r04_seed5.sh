#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 300 python -u scripts/sweep_uts.py T1 HCLIB_HIP_SPILL_LO=224,336 > gpurun_out/r04/seed5_t1.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T1L HCLIB_HIP_SPILL_LO=224,336 > gpurun_out/r04/seed5_t1l.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T1XL HCLIB_HIP_SPILL_LO=224,336 > gpurun_out/r04/seed5_t1xl.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T1XL:7 HCLIB_HIP_SPILL_LO=224,336,448 > gpurun_out/r04/seed5_t1xl7.log 2>&1 &&
timeout -k 10 300 python -u scripts/sweep_uts.py T2 HCLIB_HIP_UTS_SEED=0 > gpurun_out/r04/seed5_t2.log 2>&1 &&
timeout -k 10 300 python -u scripts/uts_probe.py T1 T1L T1XL:7 T1XL T3L fib30 > gpurun_out/r04/seed5_probe.log 2>&1 &&
echo ok
