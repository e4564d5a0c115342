set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u scripts/ab_libs.py new=hclib_amd/lib/libhclib_amd.so base=hclib_amd/lib/base/libhclib_amd.so new=hclib_amd/lib/libhclib_amd.so base=hclib_amd/lib/base/libhclib_amd.so -- T3L T1 T1L T1XL fib30 > gpurun_out/r05/ab_pend.log 2>&1; tail -8 gpurun_out/r05/ab_pend.log
