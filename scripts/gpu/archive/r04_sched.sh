#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 500 python -u scripts/ab_libs_t3l.py T3L hclib_amd/lib/libhclib_amd.so hclib_amd/lib/sched_ilp/libhclib_amd.so hclib_amd/lib/sched_minreg/libhclib_amd.so > gpurun_out/r04/sched_ab_t3l.log 2>&1 &&
timeout -k 10 400 python -u scripts/ab_libs_t3l.py T1XL hclib_amd/lib/libhclib_amd.so hclib_amd/lib/sched_ilp/libhclib_amd.so hclib_amd/lib/sched_minreg/libhclib_amd.so > gpurun_out/r04/sched_ab_t1xl.log 2>&1 &&
echo ok
