# SW-64K promise DAG: waves per CU and progressive puts
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
L=gpurun_out/sw_dag_knobs.log
: > $L
for w in 1 2 4; do
  for p in 0 1; do
    echo "== waves/CU $w progressive $p" >> $L
    SW_SCHEDS=dag SW_REPS=4 HCLIB_HIP_SW_WAVES_PER_CU=$w HCLIB_HIP_SW_PROGRESSIVE=$p timeout -k 10 120 python -u scripts/probe_sw.py 2>&1 | grep -v amdgpu.ids >> $L || exit 1
  done
done
cat $L
