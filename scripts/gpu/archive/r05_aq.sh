set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 700 python -u scripts/sweep_env.py T3L 5 '' 'HCLIB_HIP_DEQUES=128' 'HCLIB_HIP_DEQUES=256 HCLIB_HIP_DEQUE_CAP=2048' > gpurun_out/r05/sweep_dq_t3l.log 2>&1; tail -3 gpurun_out/r05/sweep_dq_t3l.log
timeout -k 10 500 python -u scripts/sweep_env.py T1XL 3 '' 'HCLIB_HIP_DEQUES=128' > gpurun_out/r05/sweep_dq_t1xl.log 2>&1; tail -2 gpurun_out/r05/sweep_dq_t1xl.log
timeout -k 10 300 python -u scripts/sweep_env.py T1 6 '' 'HCLIB_HIP_DEQUES=128' > gpurun_out/r05/sweep_dq_t1.log 2>&1; tail -2 gpurun_out/r05/sweep_dq_t1.log
