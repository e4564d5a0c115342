# fib(30): spill thresholds x chunk size at 2 waves/CU
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
L=gpurun_out/fib_knobs2.log
timeout -k 10 400 python -u scripts/sweep_uts.py fib30 HCLIB_HIP_FIB_SPILL_LO=16,32,64 HCLIB_HIP_FIB_SPILL_HI=128,256 HCLIB_HIP_FIB_CHUNK=32,64 2>&1 | grep -v amdgpu.ids > $L || exit 1
cat $L
