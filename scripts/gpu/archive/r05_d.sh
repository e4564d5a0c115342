set -o pipefail
mkdir -p gpurun_out/r05
K="sw or dag or device" TAG=sw_d bash scripts/gpu/r05_tests.sh || exit 1
timeout -k 10 300 python -u scripts/ab_libs.py early=hclib_amd/lib/libhclib_amd.so base=hclib_amd/lib/base/libhclib_amd.so -- sw_dag > gpurun_out/r05/ab_sw_early.log 2>&1; tail -4 gpurun_out/r05/ab_sw_early.log
timeout -k 10 120 python -u scripts/sw_dag_trace.py gpurun_out/r05/sw_trace.bin > gpurun_out/r05/sw_trace_early.json 2>&1; head -60 gpurun_out/r05/sw_trace_early.json
