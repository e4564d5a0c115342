set -o pipefail
mkdir -p gpurun_out/r05
HCLIB_AMD_LIB=hclib_amd/lib/phases/libhclib_amd.so HCLIB_HIP_SPILLS_PER_BATCH=1 timeout -k 10 300 python -u scripts/critpath/phases.py T3L > gpurun_out/r05/phases_sp1.jsonl 2>&1; grep tree gpurun_out/r05/phases_sp1.jsonl
timeout -k 10 600 python -u scripts/sweep_env.py T3L 5 '' 'HCLIB_HIP_SPILLS_PER_BATCH=1' 'HCLIB_HIP_SPILLS_PER_BATCH=2' 'HCLIB_HIP_HUNGER=64' > gpurun_out/r05/sweep_spills_t3l.log 2>&1; tail -4 gpurun_out/r05/sweep_spills_t3l.log
