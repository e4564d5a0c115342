set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u scripts/critpath/t3l_chain.py > gpurun_out/r05/t3l_chain.jsonl 2>&1; tail -6 gpurun_out/r05/t3l_chain.jsonl
