set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u scripts/critpath/t3l_chain.py '' > gpurun_out/r05/t3l_chain_parts.jsonl 2>&1; tail -1 gpurun_out/r05/t3l_chain_parts.jsonl
