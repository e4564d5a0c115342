set -o pipefail
mkdir -p gpurun_out/r05
HCLIB_AMD_LIB=hclib_amd/lib/phases/libhclib_amd.so timeout -k 10 300 python -u scripts/critpath/phases.py T3L T1XL T3 > gpurun_out/r05/phases.jsonl 2>&1; cat gpurun_out/r05/phases.jsonl | grep tree
