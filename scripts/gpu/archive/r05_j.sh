set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u scripts/sweep_env.py T1 3 '' 'HCLIB_HIP_SEED_PER_WAVE=64' 'HCLIB_HIP_HUNGER=16' 'HCLIB_HIP_HUNGER=8' 'HCLIB_HIP_SEED_PER_WAVE=64 HCLIB_HIP_HUNGER=16' 'HCLIB_HIP_SPILL_LO=400' > gpurun_out/r05/sweep_t1_f.log 2>&1; tail -6 gpurun_out/r05/sweep_t1_f.log
