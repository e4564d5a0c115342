set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 700 python -u scripts/sweep_env.py T3L 5 '' 'HCLIB_HIP_DEQUES=32' 'HCLIB_HIP_DEQUES=128' 'HCLIB_HIP_SPILLS_PER_BATCH=1' 'HCLIB_HIP_BACKOFF=4' > gpurun_out/r05/sweep_t3l_j.log 2>&1; tail -5 gpurun_out/r05/sweep_t3l_j.log
