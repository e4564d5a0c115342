#!/bin/bash
# T1 (small GEO tree): spill threshold / hunger interval vs the ramp-up from one root
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=10000
timeout -k 10 300 python -u scripts/sweep_uts.py T1 HCLIB_HIP_SPILL_LO=8,16,32,64,96 HCLIB_HIP_HUNGER=2,8,32 > gpurun_out/t1_ramp.log 2>&1 && echo "all ok"
