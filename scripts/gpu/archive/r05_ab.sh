set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u scripts/sweep_env.py T3 5 '' 'HCLIB_HIP_WPG=4 HCLIB_HIP_WAVES_PER_CU=4' 'HCLIB_HIP_WPG=2 HCLIB_HIP_WAVES_PER_CU=4' > gpurun_out/r05/sweep_wpg_t3.log 2>&1; tail -3 gpurun_out/r05/sweep_wpg_t3.log
timeout -k 10 600 python -u scripts/sweep_env.py T3L 5 '' 'HCLIB_HIP_WPG=4 HCLIB_HIP_WAVES_PER_CU=4' 'HCLIB_HIP_WPG=4 HCLIB_HIP_WAVES_PER_CU=4 HCLIB_HIP_SPILL_LO=72' 'HCLIB_HIP_WPG=4 HCLIB_HIP_WAVES_PER_CU=4 HCLIB_HIP_HUNGER=64' > gpurun_out/r05/sweep_wpg4_t3l.log 2>&1; tail -4 gpurun_out/r05/sweep_wpg4_t3l.log
