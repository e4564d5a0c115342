# residual of a popped range item: two halves (default) vs one whole item
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
L=gpurun_out/split_ab.log
: > $L
for v in default split3 split4 split8; do
  if [ $v = default ]; then lib=hclib_amd/lib/libhclib_amd.so; else lib=hclib_amd/lib/$v/libhclib_amd.so; fi
  for t in T1XL T1L T1 T2L T2 T4; do
    echo "== $v $t" >> $L
    HCLIB_AMD_LIB=$lib timeout -k 10 120 python -u scripts/sweep_uts.py $t 2>&1 | grep -v amdgpu.ids >> $L || exit 1
  done
done
cat $L
