set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u scripts/critpath/stress_t1.py 20 T1 T3 2>&1 | grep tree
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "uts" > gpurun_out/r05/h32_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r05/h32_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/sweep_env.py T1 6 '' 'HCLIB_HIP_HUNGER=64' > gpurun_out/r05/sweep_t1_i.log 2>&1; tail -2 gpurun_out/r05/sweep_t1_i.log
