set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u scripts/sweep_env.py T1 6 '' 'HCLIB_HIP_HUNGER=16' 'HCLIB_HIP_HUNGER=32' 'HCLIB_HIP_SPILL_LO=160' 'HCLIB_HIP_SEED_PER_WAVE=8' 'HCLIB_HIP_SEED_PER_WAVE=32' 'HCLIB_HIP_CHUNK=32' > gpurun_out/r05/sweep_t1_g.log 2>&1; tail -7 gpurun_out/r05/sweep_t1_g.log
