set -o pipefail
mkdir -p gpurun_out/r05
L=hclib_amd/lib
timeout -k 10 300 python -u scripts/critpath/stress_t1.py 20 T1 T3 T1L 2>&1 | grep tree
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05/pre_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r05/pre_tests.log; [ $rc -ne 0 ] && exit $rc
REPS=4 timeout -k 10 600 python -u scripts/ab_libs.py pre=$L/libhclib_amd.so prev=$L/prev/libhclib_amd.so -- T3L T1 T1XL fib30 > gpurun_out/r05/ab_preticket.log 2>&1; tail -8 gpurun_out/r05/ab_preticket.log
