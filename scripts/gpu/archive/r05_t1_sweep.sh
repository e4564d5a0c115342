set -o pipefail
TREES="T1" OUTF=tl_t1_b bash scripts/gpu/r05_timeline.sh &&
timeout -k 10 400 python -u scripts/sweep_env.py T1 3 '' 'HCLIB_HIP_SEED_PER_WAVE=2' 'HCLIB_HIP_SEED_PER_WAVE=1' 'HCLIB_HIP_SEED_PER_WAVE=8' 'HCLIB_HIP_WAVES_PER_CU=8' 'HCLIB_HIP_WAVES_PER_CU=8 HCLIB_HIP_SEED_PER_WAVE=2' 'HCLIB_HIP_WAVES_PER_CU=6 HCLIB_HIP_SEED_PER_WAVE=2' > gpurun_out/r05/sweep_t1_a.log 2>&1; tail -8 gpurun_out/r05/sweep_t1_a.log
