set -o pipefail
mkdir -p gpurun_out/r05
RUNS=2 timeout -k 10 300 python -u scripts/critpath/t3l_chain.py '' > gpurun_out/r05/t3l_chain_final.jsonl 2>&1; python3 scripts/critpath/summ.py gpurun_out/r05/t3l_chain_final.jsonl
