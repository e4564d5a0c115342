# fixed-shape GEO, 512-item rings: waves per CU under the new spill policy
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
L=gpurun_out/geo_waves.log
: > $L
for t in T1XL T1L; do
  echo "== $t" >> $L
  timeout -k 10 300 python -u scripts/sweep_uts.py $t HCLIB_HIP_WAVES_PER_CU=6,7,8,9 2>&1 | grep -v amdgpu.ids >> $L || exit 1
done
cat $L
