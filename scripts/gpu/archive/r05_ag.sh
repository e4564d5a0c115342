set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sw" > gpurun_out/r05/sw_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05/sw_tests.log; [ $rc -ne 0 ] && exit $rc
L=hclib_amd/lib
REPS=4 timeout -k 10 600 python -u scripts/ab_libs.py new=$L/libhclib_amd.so head=$L/headbase/libhclib_amd.so -- sw_dag sw_rows > gpurun_out/r05/ab_sw_lds.log 2>&1; tail -8 gpurun_out/r05/ab_sw_lds.log
HCLIB_AMD_LIB=$L/trace/libhclib_amd.so timeout -k 10 300 python -u scripts/sw_dag_trace.py > gpurun_out/r05/sw_trace_lds.json 2>&1; grep -A3 '"all"' gpurun_out/r05/sw_trace_lds.json | head -3; grep '"in_ingress_us"\|"in_loaded_us"\|non_sweep_per_hop' gpurun_out/r05/sw_trace_lds.json
