# after the launch-shape defaults: every published tree, then spill_lo on the small rule-table trees
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
L=gpurun_out/geo_spill5.log
: > $L
for t in T1 T2 T3 T4 T5 T1L T2L T3L T1XL; do
  echo "== $t" >> $L
  timeout -k 10 200 python -u scripts/sweep_uts.py $t 2>&1 | grep -v amdgpu.ids >> $L || exit 1
done
for t in T2 T5 T4; do
  echo "== $t spill_lo at 4 waves/CU" >> $L
  timeout -k 10 200 python -u scripts/sweep_uts.py $t HCLIB_HIP_SPILL_LO=96,160,224,336 2>&1 | grep -v amdgpu.ids >> $L || exit 1
done
cat $L
