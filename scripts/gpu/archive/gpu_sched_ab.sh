# A/B of LLVM AMDGPU machine-scheduler strategies on the UTS/fib kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
L=gpurun_out/sched_ab.log
: > $L
for v in default sched_minreg sched_ilp; do
  if [ $v = default ]; then lib=hclib_amd/lib/libhclib_amd.so; else lib=hclib_amd/lib/$v/libhclib_amd.so; fi
  for t in T3L T1XL fib30; do
    echo "== $v $t" >> $L
    HCLIB_AMD_LIB=$lib timeout -k 10 120 python -u scripts/sweep_uts.py $t >> $L 2>&1 || exit 1
  done
done
cat $L
