# T3L: number of HBM deques x chunk size
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/sweep_uts.py T3L HCLIB_HIP_DEQUES=16,32,64,128 HCLIB_HIP_CHUNK=32,64 2>&1 | grep -v amdgpu.ids > gpurun_out/t3l_deques.log || exit 1
cat gpurun_out/t3l_deques.log
