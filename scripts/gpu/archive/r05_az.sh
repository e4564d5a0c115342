set -o pipefail
mkdir -p gpurun_out/r05
for h in 64 128; do HCLIB_HIP_HUNGER=$h timeout -k 10 400 python -u scripts/shard_ab.py 3 h$h=hclib_amd/lib/libhclib_amd.so 2>&1 | tail -1 | cut -c1-300; done
