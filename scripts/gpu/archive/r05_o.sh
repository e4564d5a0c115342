set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u scripts/t3l_bands.py --band 2000 > gpurun_out/r05/t3l_bands.jsonl 2>&1; tail -12 gpurun_out/r05/t3l_bands.jsonl
