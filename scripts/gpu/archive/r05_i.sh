set -o pipefail
mkdir -p gpurun_out/r05
K="uts" TAG=uts_i bash scripts/gpu/r05_tests.sh || exit 1
timeout -k 10 600 python -u scripts/sweep_env.py T1 3 '' 'HCLIB_HIP_WAVES_PER_CU=4' 'HCLIB_HIP_SEED_PER_WAVE=8' > gpurun_out/r05/sweep_t1_e.log 2>&1; tail -3 gpurun_out/r05/sweep_t1_e.log
timeout -k 10 600 python -u scripts/sweep_env.py T1XL 2 '' 'HCLIB_HIP_SEED_PER_WAVE=16' 'HCLIB_HIP_SEED_PER_WAVE=48' > gpurun_out/r05/sweep_t1xl_e.log 2>&1; tail -3 gpurun_out/r05/sweep_t1xl_e.log
