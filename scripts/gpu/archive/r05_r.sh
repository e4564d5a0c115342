set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u scripts/ab_libs.py nap=hclib_amd/lib/libhclib_amd.so nonap=hclib_amd/lib/nonap/libhclib_amd.so -- T3L T1 > gpurun_out/r05/ab_nap.log 2>&1; tail -6 gpurun_out/r05/ab_nap.log
timeout -k 10 300 python -u scripts/critpath/t3l_chain.py '' > gpurun_out/r05/t3l_chain_nap.jsonl 2>&1; tail -1 gpurun_out/r05/t3l_chain_nap.jsonl | cut -c1-900
