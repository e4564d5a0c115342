set -o pipefail
mkdir -p gpurun_out/r05
L=hclib_amd/lib
REPS=4 timeout -k 10 600 python -u scripts/ab_libs.py new=$L/libhclib_amd.so head=$L/headbase/libhclib_amd.so -- T3L T1 T1XL fib30 > gpurun_out/r05/ab_waits.log 2>&1; tail -8 gpurun_out/r05/ab_waits.log
timeout -k 10 300 python -u scripts/critpath/t3l_chain.py '' > gpurun_out/r05/t3l_chain_waits.jsonl 2>&1; python3 scripts/critpath/summ.py gpurun_out/r05/t3l_chain_waits.jsonl
