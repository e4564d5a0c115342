# cross-GPU sharing region in each memory kind: rehearsal (2 ranks, one GPU) + GPU test
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export HCLIB_HIP_SPIN_LIMIT_MS=10000
# two persistent kernels share one GPU here: each must leave room for the other
# to be resident (on N GPUs each rank has its own)
export HCLIB_HIP_WAVES_PER_CU=2
for k in ${KINDS:-uncached fine device}; do
  echo "== $k"
  HCLIB_GLOBAL_MEM=$k REHEARSE_CASES="T1L:1,T3L:64" timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 2955$((RANDOM % 10)) scripts/rehearse_global.py || echo "FAILED $k"
done > gpurun_out/global_mem_kinds.log 2>&1
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu.py -k "sharing" > gpurun_out/global_test.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/global_mem_kinds.log; tail -5 gpurun_out/global_test.log; exit $rc
