set -o pipefail
K="shards or partition or bench_launch" TAG=uts_g bash scripts/gpu/r05_tests.sh
for o in fwd rev; do ORDER=$o SPLIT=7 timeout -k 10 300 python -u scripts/shard_ab.py 2 new=hclib_amd/lib/libhclib_amd.so; ORDER=$o SPLIT=8 timeout -k 10 300 python -u scripts/shard_ab.py 2 new=hclib_amd/lib/libhclib_amd.so; done > gpurun_out/r05/shard_order.log 2>&1; cat gpurun_out/r05/shard_order.log
bash scripts/gpu/r05_f.sh
