#!/bin/bash
# cross-GPU sharing: the GPU test, then bench.py's N=2 form rehearsed on one GPU (gloo)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -x -q --timeout 150 --timeout-method thread -k "cross_gpu" > gpurun_out/global_test.log 2>&1 && echo "test ok" &&
HCLIB_HIP_WAVES_PER_CU=2 HCLIB_HIP_SPIN_LIMIT_MS=10000 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --backend gloo --share-device > gpurun_out/bench_n2_rehearsal.json 2> gpurun_out/bench_n2_rehearsal.err && echo "n2 rehearsal ok"
