set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u scripts/sweep_env.py T1 3 '' 'HCLIB_HIP_WAVES_PER_CU=8 HCLIB_HIP_SEED_PER_WAVE=8' 'HCLIB_HIP_WAVES_PER_CU=8 HCLIB_HIP_SEED_PER_WAVE=16' 'HCLIB_HIP_WAVES_PER_CU=8 HCLIB_HIP_SEED_PER_WAVE=4' 'HCLIB_HIP_WAVES_PER_CU=6 HCLIB_HIP_SEED_PER_WAVE=8' 'HCLIB_HIP_WAVES_PER_CU=4 HCLIB_HIP_SEED_PER_WAVE=16' 'HCLIB_HIP_WAVES_PER_CU=8 HCLIB_HIP_SEED_PER_WAVE=8 HCLIB_HIP_SPILL_LO=448' 'HCLIB_HIP_WAVES_PER_CU=8 HCLIB_HIP_SEED_PER_WAVE=8 HCLIB_HIP_SPILL_LO=256' > gpurun_out/r05/sweep_t1_d.log 2>&1; tail -8 gpurun_out/r05/sweep_t1_d.log
timeout -k 10 300 python -u scripts/sweep_env.py T1L 2 '' 'HCLIB_HIP_SEED_PER_WAVE=16' 'HCLIB_HIP_SEED_PER_WAVE=64' > gpurun_out/r05/sweep_t1l_d.log 2>&1; tail -3 gpurun_out/r05/sweep_t1l_d.log
