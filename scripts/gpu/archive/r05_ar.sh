set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u scripts/critpath/stress_t1.py 15 T1 T3 2>&1 | grep tree
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05/dq_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r05/dq_tests.log; exit $rc
