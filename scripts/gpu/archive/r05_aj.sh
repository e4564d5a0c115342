set -o pipefail
mkdir -p gpurun_out/r05
L=hclib_amd/lib
echo new; timeout -k 10 200 python -u scripts/critpath/stress_t1.py 30 T1 T3 2>&1 | grep tree
echo prev; HCLIB_AMD_LIB=$L/prev/libhclib_amd.so timeout -k 10 200 python -u scripts/critpath/stress_t1.py 30 T1 T3 2>&1 | grep tree
