set -o pipefail
mkdir -p gpurun_out/r05
L=hclib_amd/lib
timeout -k 10 500 python -u scripts/ab_libs.py new=$L/libhclib_amd.so base=$L/r05base/libhclib_amd.so nonap=$L/nonap/libhclib_amd.so spill1=$L/spill1/libhclib_amd.so late0=$L/late0/libhclib_amd.so -- T3L T1 T1XL fib30 > gpurun_out/r05/ab_idle3.log 2>&1; tail -10 gpurun_out/r05/ab_idle3.log
timeout -k 10 300 python -u scripts/critpath/t3l_chain.py '' 'HCLIB_HIP_DEFER=0' > gpurun_out/r05/t3l_chain_new.jsonl 2>&1; tail -2 gpurun_out/r05/t3l_chain_new.jsonl | cut -c1-1200
