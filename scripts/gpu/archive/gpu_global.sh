#!/bin/bash
# cross-GPU work sharing rehearsal: 2 ranks on one GPU (gloo, IPC-mapped region)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=10000 HCLIB_HIP_WAVES_PER_CU=2
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 scripts/rehearse_global.py > gpurun_out/global_rehearsal.log 2> gpurun_out/global_rehearsal.err && echo "global rehearsal ok"
