set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 500 python -u scripts/shard_ab.py 3 final=hclib_amd/lib/libhclib_amd.so > gpurun_out/r05/shard_final.log 2>&1; tail -3 gpurun_out/r05/shard_final.log | cut -c1-600
