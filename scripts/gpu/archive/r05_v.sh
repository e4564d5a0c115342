set -o pipefail
mkdir -p gpurun_out/r05
HCLIB_AMD_LIB=hclib_amd/lib/stamps/libhclib_amd.so timeout -k 10 300 python -u scripts/probe_stamps.py > gpurun_out/r05/stamps_t3l.log 2>&1; head -4 gpurun_out/r05/stamps_t3l.log
