# GEO 512-item rings: children pushed as 3, 2 or 1 range items; spill_lo at 3 pieces
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
L=gpurun_out/pieces_ab2.log
: > $L
for v in pieces3 pieces2 pieces1; do
  lib=hclib_amd/lib/$v/libhclib_amd.so
  for t in T1XL T1L T2L T2 T5 T4; do
    echo "== $v $t" >> $L
    HCLIB_AMD_LIB=$lib timeout -k 10 120 python -u scripts/sweep_uts.py $t 2>&1 | grep -v amdgpu.ids >> $L || exit 1
  done
done
for t in T1XL T1L; do
  echo "== pieces3 $t spill_lo" >> $L
  HCLIB_AMD_LIB=hclib_amd/lib/pieces3/libhclib_amd.so timeout -k 10 200 python -u scripts/sweep_uts.py $t HCLIB_HIP_SPILL_LO=224,336,416 2>&1 | grep -v amdgpu.ids >> $L || exit 1
done
cat $L
