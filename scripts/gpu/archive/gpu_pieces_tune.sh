# fixed-shape GEO at one piece per task: UTS parity tests, then spill_lo / hunger / waves
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "uts" > gpurun_out/uts_tests.log 2>&1 || { tail -30 gpurun_out/uts_tests.log; exit 1; }
tail -2 gpurun_out/uts_tests.log
L=gpurun_out/pieces_tune.log
: > $L
for t in T1XL T1L; do
  echo "== $t" >> $L
  timeout -k 10 300 python -u scripts/sweep_uts.py $t HCLIB_HIP_SPILL_LO=160,224,336,448 HCLIB_HIP_HUNGER=32,64 2>&1 | grep -v amdgpu.ids >> $L || exit 1
  timeout -k 10 300 python -u scripts/sweep_uts.py $t HCLIB_HIP_WAVES_PER_CU=8,9,10 2>&1 | grep -v amdgpu.ids >> $L || exit 1
done
cat $L
