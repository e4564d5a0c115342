set -o pipefail
mkdir -p gpurun_out/r05
K="uts" TAG=uts_m bash scripts/gpu/r05_tests.sh || exit 1
timeout -k 10 900 python -u scripts/ab_libs.py new=hclib_amd/lib/libhclib_amd.so base=hclib_amd/lib/base/libhclib_amd.so new=hclib_amd/lib/libhclib_amd.so base=hclib_amd/lib/base/libhclib_amd.so new=hclib_amd/lib/libhclib_amd.so base=hclib_amd/lib/base/libhclib_amd.so -- T3L T1XL > gpurun_out/r05/ab_inbox.log 2>&1; tail -8 gpurun_out/r05/ab_inbox.log
