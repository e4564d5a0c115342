#!/bin/bash
# A/B in one process lifetime each, interleaved: inline (default) vs noinline narrow loop
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
  timeout -k 10 120 python -u scripts/sweep_uts.py T3L HCLIB_HIP_SPILL_LO=72,96 | sed 's/^/noinline /' || exit 1
  HCLIB_AMD_LIB=hclib_amd/lib/narrow_noinline/libhclib_amd.so timeout -k 10 120 python -u scripts/sweep_uts.py T3L HCLIB_HIP_SPILL_LO=72,96 | sed 's/^/inline   /' || exit 1
done
