set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u scripts/ab_libs.py base=hclib_amd/lib/libhclib_amd.so excess=hclib_amd/lib/excess/libhclib_amd.so base=hclib_amd/lib/libhclib_amd.so excess=hclib_amd/lib/excess/libhclib_amd.so -- T3L > gpurun_out/r05/ab_excess.log 2>&1; tail -8 gpurun_out/r05/ab_excess.log
HCLIB_AMD_LIB=hclib_amd/lib/excess/libhclib_amd.so timeout -k 10 600 python -u scripts/sweep_env.py T3L 2 'HCLIB_HIP_SPILL_LO=65' 'HCLIB_HIP_SPILL_LO=80' 'HCLIB_HIP_SPILL_LO=96' > gpurun_out/r05/sweep_excess.log 2>&1; tail -3 gpurun_out/r05/sweep_excess.log
