#!/bin/bash
# Round-3 GPU pass: dual-chain SHA-1 ubench, parity suite, the bench line under
# rocprofv3 kernel-trace (bench.json + kernel stats of the SAME command), the
# triad PMC passes, the CPU-port thread sweep. Each GPU step has its own limit;
# steps chained with &&. usage: scripts/gpu_r03.sh OUTDIR [steps...]
# steps: ub valu bands ab tests bench pmc sweep (default: all)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r03}; shift
STEPS=${*:-ub ab tests bench pmc sweep}
mkdir -p $OUT
has() { [[ " $STEPS " == *" $1 "* ]]; }
if has ub; then
  timeout -k 10 120 scripts/ubench/ub_sha2.bin > $OUT/ub_sha2.log 2>&1 || { echo "ub failed"; exit 1; }
  cat $OUT/ub_sha2.log
fi
if has valu; then
  timeout -k 10 120 scripts/ubench/ub_valu.bin > $OUT/ub_valu.log 2>&1 || { echo "valu failed"; exit 1; }
  cat $OUT/ub_valu.log
fi
if has bands; then
  timeout -k 10 300 python -u scripts/t3l_bands.py > $OUT/t3l_bands.jsonl 2> $OUT/t3l_bands.err || { echo "bands failed"; tail -20 $OUT/t3l_bands.err; exit 1; }
  cat $OUT/t3l_bands.jsonl
fi
if has ab; then
  for T in T1XL T1L T1; do
    timeout -k 10 200 python -u scripts/sweep_uts.py $T HCLIB_HIP_UTS_DUAL=0,1,0,1 >> $OUT/dual_ab.log 2>&1 || { echo "ab failed"; tail -20 $OUT/dual_ab.log; exit 1; }
  done
  cat $OUT/dual_ab.log
fi
if has tests; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -3 $OUT/gpu_tests.log
fi
if has bench; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/prof -o run -- python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
if has pmc; then
  mkdir -p $OUT/pmc
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc/fetch -o f -- python3 scripts/triad_pmc_run.py > $OUT/pmc/fetch.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc/write -o w -- python3 scripts/triad_pmc_run.py > $OUT/pmc/write.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $OUT/pmc/req -o r -- python3 scripts/triad_pmc_run.py > $OUT/pmc/req.log 2>&1 || { echo "pmc failed"; exit 1; }
  echo "pmc ok"
fi
if has sweep; then
  timeout -k 10 400 python3 scripts/cpu_thread_sweep.py > $OUT/cpu_sweep.json 2> $OUT/cpu_sweep.log || { echo "sweep failed"; cat $OUT/cpu_sweep.log; exit 1; }
  cat $OUT/cpu_sweep.log
fi
echo "all ok"
