# fixed-shape GEO, one piece per task: spill_hi x chunk
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
L=gpurun_out/geo_hi.log
: > $L
for t in T1XL T1L; do
  echo "== $t" >> $L
  timeout -k 10 300 python -u scripts/sweep_uts.py $t HCLIB_HIP_SPILL_HI=384,448,512 HCLIB_HIP_CHUNK=32,64 2>&1 | grep -v amdgpu.ids >> $L || exit 1
done
cat $L
