set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 500 python -u scripts/critpath/t3l_chain.py '' 'HCLIB_HIP_DEFER=0' 'HCLIB_HIP_BACKOFF=4' 'HCLIB_HIP_BACKOFF=1' 'HCLIB_HIP_WPG=4 HCLIB_HIP_WAVES_PER_CU=4' 'HCLIB_HIP_CHUNK=32' 'HCLIB_HIP_WAVES_PER_CU=4' > gpurun_out/r05/t3l_chain_cfg.jsonl 2>&1; tail -3 gpurun_out/r05/t3l_chain_cfg.jsonl | cut -c1-300
