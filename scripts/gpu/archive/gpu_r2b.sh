#!/bin/bash
# round 2: UTS diagnostics — T1XL PMC passes, per-phase stamps (diagnostic build), T1 default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=10000
bash scripts/pmc_uts.sh T1XL 0 gpurun_out/pmc_t1xl > gpurun_out/pmc_t1xl.log 2>&1 && echo "pmc ok" &&
python3 scripts/pmc_summary.py gpurun_out/pmc_t1xl > gpurun_out/pmc_t1xl_summary.txt &&
HCLIB_AMD_LIB=hclib_amd/lib/stamps/libhclib_amd.so timeout -k 10 300 python -u scripts/probe_stamps.py > gpurun_out/stamps.log 2>&1 && echo "stamps ok" &&
timeout -k 10 200 python -u scripts/sweep_uts.py T1 HCLIB_HIP_CARRY=1 > gpurun_out/t1_default.log 2>&1 && echo "all ok"
