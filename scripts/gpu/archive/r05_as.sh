set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u scripts/critpath/fib_env.py 8 '' 'HCLIB_HIP_DEQUES=128' 'HCLIB_HIP_DEQUES=32' 'HCLIB_HIP_WAVES_PER_CU=4' 'HCLIB_HIP_WAVES_PER_CU=2' > gpurun_out/r05/fib_env.log 2>&1; cat gpurun_out/r05/fib_env.log | grep fib30
timeout -k 10 500 python -u scripts/sweep_env.py T1XL 3 '' 'HCLIB_HIP_HUNGER=96' 'HCLIB_HIP_SPILL_LO=288' > gpurun_out/r05/sweep_t1xl_k.log 2>&1; tail -3 gpurun_out/r05/sweep_t1xl_k.log
