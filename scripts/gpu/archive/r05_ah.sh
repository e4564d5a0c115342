set -o pipefail
HCLIB_AMD_LIB=hclib_amd/lib/phases/libhclib_amd.so timeout -k 10 300 python -u scripts/critpath/phases.py T3L 2>&1 | grep tree
