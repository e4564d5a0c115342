set -o pipefail
mkdir -p gpurun_out/r05
L0=hclib_amd/lib/late0/libhclib_amd.so
timeout -k 10 400 python -u scripts/sweep_env.py T3L 6 '' 'HCLIB_HIP_DEFER=0' "HCLIB_AMD_LIB=$L0" "HCLIB_AMD_LIB=$L0 HCLIB_HIP_DEFER=0" > gpurun_out/r05/sweep_defer_t3l.log 2>&1; tail -4 gpurun_out/r05/sweep_defer_t3l.log
timeout -k 10 300 python -u scripts/sweep_env.py T1XL 3 '' 'HCLIB_HIP_DEFER=0' "HCLIB_AMD_LIB=$L0" "HCLIB_AMD_LIB=$L0 HCLIB_HIP_DEFER=0" > gpurun_out/r05/sweep_defer_t1xl.log 2>&1; tail -4 gpurun_out/r05/sweep_defer_t1xl.log
timeout -k 10 300 python -u scripts/sweep_env.py T1 4 '' 'HCLIB_HIP_DEFER=0' "HCLIB_AMD_LIB=$L0" "HCLIB_AMD_LIB=$L0 HCLIB_HIP_DEFER=0" > gpurun_out/r05/sweep_defer_t1.log 2>&1; tail -4 gpurun_out/r05/sweep_defer_t1.log
