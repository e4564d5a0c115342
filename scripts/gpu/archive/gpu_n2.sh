#!/bin/bash
# N=2 rehearsal on one GPU (gloo, both ranks on device 0): bench.py's N>1 form
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
# both ranks' persistent grids must be resident together on the one GPU
# (DESIGN §6): 2 waves per CU each
export HCLIB_HIP_WAVES_PER_CU=2
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --backend gloo --share-device > gpurun_out/bench_n2_rehearsal.json 2> gpurun_out/bench_n2_rehearsal.err && echo "n2 rehearsal ok"
