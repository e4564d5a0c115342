set -o pipefail
mkdir -p gpurun_out/r05
K=uts TAG=uts_b bash scripts/gpu/r05_tests.sh || exit 1
timeout -k 10 300 python -u scripts/shard_ab.py 2 new=hclib_amd/lib/libhclib_amd.so loop=hclib_amd/lib/shardloop/libhclib_amd.so new=hclib_amd/lib/libhclib_amd.so loop=hclib_amd/lib/shardloop/libhclib_amd.so > gpurun_out/r05/shard_ab.log 2>&1; cat gpurun_out/r05/shard_ab.log
bash scripts/gpu/r05_t1_sweep2.sh
