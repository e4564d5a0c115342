#!/bin/bash
# GPU pass for the sharded SW path: band parity tests, then the full GPU
# suite, then a 2-rank shared-device bench rehearsal (gloo, both ranks on
# cuda:0). Every GPU step has its own time limit; steps chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_gpu.py -x -v -m gpu -k "band or sharded" --timeout 120 --timeout-method thread > gpurun_out/swband_tests.log 2>&1 && echo "band tests ok" &&
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo "gpu tests ok" &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 0 --backend gloo --share-device > gpurun_out/bench_n2_rehearsal.json 2> gpurun_out/bench_n2_rehearsal.err && echo "n2 rehearsal ok"
