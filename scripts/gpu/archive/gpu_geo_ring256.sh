# fixed-shape GEO: 256-item rings (8 KiB per wave) for large trees now that 512 rings also run one piece per task
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
L=gpurun_out/geo_ring256.log
: > $L
for t in T1XL T1L; do
  echo "== $t ring 256" >> $L
  HCLIB_HIP_UTS_RING=256 timeout -k 10 300 python -u scripts/sweep_uts.py $t HCLIB_HIP_WAVES_PER_CU=8,12 HCLIB_HIP_SPILL_LO=128,192 HCLIB_HIP_SPILL_HI=224,512 2>&1 | grep -v amdgpu.ids >> $L || exit 1
done
cat $L
