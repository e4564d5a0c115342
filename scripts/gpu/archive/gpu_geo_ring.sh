# fixed-shape GEO: 1024-item rings (8 pieces) vs the 512 default under the new spill policy
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
L=gpurun_out/geo_ring.log
: > $L
for t in T1XL T1L; do
  echo "== $t ring 1024" >> $L
  HCLIB_HIP_UTS_RING=1024 timeout -k 10 300 python -u scripts/sweep_uts.py $t HCLIB_HIP_WAVES_PER_CU=4,5 HCLIB_HIP_SPILL_LO=336,640 HCLIB_HIP_SPILL_HI=512,960 2>&1 | grep -v amdgpu.ids >> $L || exit 1
done
cat $L
