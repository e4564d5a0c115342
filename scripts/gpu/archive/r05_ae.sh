set -o pipefail
mkdir -p gpurun_out/r05
for sp in 0 1; do HCLIB_AMD_LIB=hclib_amd/lib/phases/libhclib_amd.so HCLIB_HIP_SPILLS_PER_BATCH=$sp timeout -k 10 300 python -u scripts/critpath/phases.py T3L 2>&1 | grep tree; done
