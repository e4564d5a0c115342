set -o pipefail
mkdir -p gpurun_out/r05
L=hclib_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "uts" > gpurun_out/r05/excess_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05/excess_tests.log; [ $rc -ne 0 ] && exit $rc
REPS=3 timeout -k 10 600 python -u scripts/ab_libs.py excess=$L/libhclib_amd.so noexcess=$L/noexcess/libhclib_amd.so ring128=$L/ringmax128/libhclib_amd.so -- T3L T1 T1XL > gpurun_out/r05/ab_excess2.log 2>&1; tail -9 gpurun_out/r05/ab_excess2.log
timeout -k 10 300 python -u scripts/critpath/t3l_chain.py '' > gpurun_out/r05/t3l_chain_excess.jsonl 2>&1; python3 scripts/critpath/summ.py gpurun_out/r05/t3l_chain_excess.jsonl
