set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 500 python -u scripts/critpath/t3l_chain.py '' 'HCLIB_HIP_WPG=4 HCLIB_HIP_WAVES_PER_CU=4' 'HCLIB_HIP_WPG=4 HCLIB_HIP_WAVES_PER_CU=4 HCLIB_HIP_SPILL_LO=80' 'HCLIB_HIP_WAVES_PER_CU=3 HCLIB_HIP_WPG=1' > gpurun_out/r05/t3l_chain_wpg.jsonl 2>&1; python3 scripts/critpath/summ.py gpurun_out/r05/t3l_chain_wpg.jsonl
