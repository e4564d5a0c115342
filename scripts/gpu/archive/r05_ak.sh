set -o pipefail
mkdir -p gpurun_out/r05
L=hclib_amd/lib
timeout -k 10 300 python -u scripts/critpath/stress_t1.py 30 T1 T3 T1L 2>&1 | grep tree
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "uts or fib" > gpurun_out/r05/spill_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r05/spill_tests.log; [ $rc -ne 0 ] && exit $rc
HCLIB_AMD_LIB=hclib_amd/lib/phases/libhclib_amd.so timeout -k 10 300 python -u scripts/critpath/phases.py T3L 2>&1 | grep tree
REPS=4 timeout -k 10 600 python -u scripts/ab_libs.py new=$L/libhclib_amd.so prev=$L/prev/libhclib_amd.so -- T3L T1 T1XL fib30 > gpurun_out/r05/ab_spillpath.log 2>&1; tail -8 gpurun_out/r05/ab_spillpath.log
