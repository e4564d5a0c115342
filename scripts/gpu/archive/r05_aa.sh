set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 700 python -u scripts/sweep_env.py T3L 6 '' 'HCLIB_HIP_WPG=4 HCLIB_HIP_WAVES_PER_CU=4' 'HCLIB_HIP_WPG=2 HCLIB_HIP_WAVES_PER_CU=4' > gpurun_out/r05/sweep_wpg_t3l.log 2>&1; tail -4 gpurun_out/r05/sweep_wpg_t3l.log
