set -o pipefail
mkdir -p gpurun_out/r05
G=hclib_amd/lib/gate/libhclib_amd.so
timeout -k 10 600 python -u scripts/sweep_env.py T1 3 '' "HCLIB_AMD_LIB=$G" "HCLIB_AMD_LIB=$G HCLIB_HIP_SPILL_LO=224" "HCLIB_AMD_LIB=$G HCLIB_HIP_SPILL_LO=128" "HCLIB_AMD_LIB=$G HCLIB_HIP_SPILL_LO=96" > gpurun_out/r05/sweep_gate_t1.log 2>&1; tail -5 gpurun_out/r05/sweep_gate_t1.log
timeout -k 10 600 python -u scripts/sweep_env.py T1XL 2 '' "HCLIB_AMD_LIB=$G" "HCLIB_AMD_LIB=$G HCLIB_HIP_SPILL_LO=224" > gpurun_out/r05/sweep_gate_t1xl.log 2>&1; tail -3 gpurun_out/r05/sweep_gate_t1xl.log
timeout -k 10 600 python -u scripts/sweep_env.py T3L 2 '' "HCLIB_AMD_LIB=$G" > gpurun_out/r05/sweep_gate_t3l.log 2>&1; tail -2 gpurun_out/r05/sweep_gate_t3l.log
timeout -k 10 600 python -u scripts/sweep_env.py T3L 2 '' 'HCLIB_HIP_BACKOFF=32' 'HCLIB_HIP_BACKOFF=64' > gpurun_out/r05/sweep_backoff_t3l.log 2>&1; tail -3 gpurun_out/r05/sweep_backoff_t3l.log
