set -o pipefail
mkdir -p gpurun_out/r05
L=hclib_amd/lib
REPS=4 timeout -k 10 800 python -u scripts/ab_libs.py new=$L/libhclib_amd.so head=$L/headbase/libhclib_amd.so nonap=$L/nonap/libhclib_amd.so noafter=$L/noafter/libhclib_amd.so noasmst=$L/noasmst/libhclib_amd.so nodrain=$L/nodrain/libhclib_amd.so -- T3L T1XL > gpurun_out/r05/ab_bisect.log 2>&1; tail -24 gpurun_out/r05/ab_bisect.log
