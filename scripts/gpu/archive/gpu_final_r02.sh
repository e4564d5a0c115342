# final round-2 pass: full GPU suite, bench, kernel stats, T1 ring check, T1XL PMC
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
bash scripts/gpu_round2.sh || exit 1
timeout -k 10 200 python -u scripts/sweep_uts.py T1 HCLIB_HIP_UTS_RING=256,512 2>&1 | grep -v amdgpu.ids > gpurun_out/t1_ring.log || exit 1
cat gpurun_out/t1_ring.log
bash scripts/pmc_uts.sh T1XL 0 gpurun_out/pmc_t1xl_s10
