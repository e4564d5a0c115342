set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u scripts/sweep_env.py T3L 7 '' 'HCLIB_HIP_HUNGER=64' 'HCLIB_HIP_SPILLS_PER_BATCH=1' 'HCLIB_HIP_HUNGER=64 HCLIB_HIP_SPILLS_PER_BATCH=1' > gpurun_out/r05/sweep_h64sp1_t3l.log 2>&1; tail -4 gpurun_out/r05/sweep_h64sp1_t3l.log
