set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u scripts/sweep_env.py T1 8 '' 'HCLIB_HIP_HUNGER=24' 'HCLIB_HIP_HUNGER=32' 'HCLIB_HIP_HUNGER=48' > gpurun_out/r05/sweep_t1_h.log 2>&1; tail -4 gpurun_out/r05/sweep_t1_h.log
timeout -k 10 400 python -u scripts/sweep_env.py T1L 4 '' 'HCLIB_HIP_HUNGER=32' > gpurun_out/r05/sweep_t1l_h.log 2>&1; tail -2 gpurun_out/r05/sweep_t1l_h.log
