set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u scripts/ab_libs.py fence=hclib_amd/lib/libhclib_amd.so nofence=hclib_amd/lib/seedfence0/libhclib_amd.so -- T1 T1L > gpurun_out/r05/ab_seedfence.log 2>&1; tail -4 gpurun_out/r05/ab_seedfence.log
timeout -k 10 500 python -u scripts/sweep_env.py T1 3 '' 'HCLIB_HIP_SEED_PER_WAVE=16' 'HCLIB_HIP_SEED_PER_WAVE=48' 'HCLIB_HIP_SEED_PER_WAVE=16 HCLIB_HIP_SPILL_LO=224' 'HCLIB_HIP_SEED_PER_WAVE=16 HCLIB_HIP_SPILL_LO=128' 'HCLIB_HIP_SEED_PER_WAVE=16 HCLIB_HIP_WAVES_PER_CU=8' 'HCLIB_HIP_SEED_PER_WAVE=16 HCLIB_HIP_WAVES_PER_CU=6' > gpurun_out/r05/sweep_t1_b.log 2>&1; tail -8 gpurun_out/r05/sweep_t1_b.log
bash scripts/pmc_atomics_r05.sh > gpurun_out/r05/pmc_atomics.log 2>&1; tail -2 gpurun_out/r05/pmc_atomics.log
