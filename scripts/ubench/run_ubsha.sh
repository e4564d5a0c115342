# SHA-1 step latency under each LLVM AMDGPU scheduler strategy. Build first (CPU):
#   for s in default max-ilp iterative-ilp iterative-maxocc iterative-minreg; do
#     F=$([ $s = default ] || echo "-mllvm -amdgpu-sched-strategy=$s")
#     hipcc --offload-arch=gfx950 -O3 -ffp-contract=off $F scripts/ubench/ub_sha_split.hip -o scripts/ubench/ubsha_$s; done
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for s in default max-ilp iterative-ilp iterative-maxocc iterative-minreg; do echo "== $s"; timeout -k 5 60 scripts/ubench/ubsha_$s | grep -E "one-wave|rounds" ; done > gpurun_out/ubsha_sched.log 2>&1
cat gpurun_out/ubsha_sched.log
