set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 800 python -u scripts/sweep_env.py T3L 5 '' 'HCLIB_HIP_CHUNK=32' 'HCLIB_HIP_CHUNK=48' 'HCLIB_HIP_BACKOFF=8' > gpurun_out/r05/sweep_t3l_m.log 2>&1; tail -4 gpurun_out/r05/sweep_t3l_m.log
