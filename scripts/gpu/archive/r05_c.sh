set -o pipefail
mkdir -p gpurun_out/r05
for sp in 7 8 9 10; do SPLIT=$sp timeout -k 10 300 python -u scripts/shard_ab.py 2 new=hclib_amd/lib/libhclib_amd.so; done > gpurun_out/r05/shard_split.log 2>&1; cat gpurun_out/r05/shard_split.log
timeout -k 10 300 python -u scripts/sweep_env.py T1 3 '' 'HCLIB_HIP_SEED_PER_WAVE=16' 'HCLIB_HIP_SEED_PER_WAVE=2' 'HCLIB_HIP_WAVES_PER_CU=8 HCLIB_HIP_SEED_PER_WAVE=8' > gpurun_out/r05/sweep_t1_c.log 2>&1; tail -4 gpurun_out/r05/sweep_t1_c.log
