set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u scripts/sweep_env.py T1XL 4 '' 'HCLIB_HIP_HUNGER=96' 'HCLIB_HIP_HUNGER=128' 'HCLIB_HIP_HUNGER=192' > gpurun_out/r05/sweep_t1xl_l.log 2>&1; tail -4 gpurun_out/r05/sweep_t1xl_l.log
timeout -k 10 300 python -u scripts/sweep_env.py T1L 5 '' 'HCLIB_HIP_HUNGER=96' 'HCLIB_HIP_HUNGER=128' > gpurun_out/r05/sweep_t1l_l.log 2>&1; tail -3 gpurun_out/r05/sweep_t1l_l.log
