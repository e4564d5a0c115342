# BIN trees: T3 (small, critical q*m) and T3L launch shape
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
L=gpurun_out/bin_knobs.log
: > $L
echo "== T3" >> $L
timeout -k 10 300 python -u scripts/sweep_uts.py T3 HCLIB_HIP_WAVES_PER_CU=2,4,8 HCLIB_HIP_SPILL_LO=72,128,224 2>&1 | grep -v amdgpu.ids >> $L || exit 1
echo "== T3 hunger" >> $L
timeout -k 10 300 python -u scripts/sweep_uts.py T3 HCLIB_HIP_HUNGER=8,32,64 2>&1 | grep -v amdgpu.ids >> $L || exit 1
echo "== T3L spill_lo / hunger" >> $L
timeout -k 10 300 python -u scripts/sweep_uts.py T3L HCLIB_HIP_SPILL_LO=72,96 HCLIB_HIP_HUNGER=16,32,64 2>&1 | grep -v amdgpu.ids >> $L || exit 1
cat $L
