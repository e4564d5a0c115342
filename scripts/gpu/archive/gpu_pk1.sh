set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pk1
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "packed_half or generic_promise_dag or both_schedules" > gpurun_out/pk1/tests.log 2>&1 || { tail -30 gpurun_out/pk1/tests.log; exit 1; }
tail -15 gpurun_out/pk1/tests.log
timeout -k 10 200 python -u scripts/sw_pk_ab.py 3 > gpurun_out/pk1/ab.log 2>&1 || { tail -20 gpurun_out/pk1/ab.log; exit 1; }
cat gpurun_out/pk1/ab.log
