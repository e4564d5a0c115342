# T1XL: hunger interval around 64 (spill defaults of 33e41c3), twice for spread
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
L=gpurun_out/geo_knobs2.log
: > $L
for rep in 1 2; do
  echo "== T1XL pass $rep" >> $L
  timeout -k 10 300 python -u scripts/sweep_uts.py T1XL HCLIB_HIP_HUNGER=32,48,64,96,128 2>&1 | grep -v amdgpu.ids >> $L || exit 1
done
echo "== T1L" >> $L
timeout -k 10 300 python -u scripts/sweep_uts.py T1L HCLIB_HIP_HUNGER=32,64,96 2>&1 | grep -v amdgpu.ids >> $L || exit 1
cat $L
