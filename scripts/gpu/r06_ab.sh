#!/bin/bash
# round 6: UTS GPU tests (K filter), then an interleaved A/B of the base
# library (hclib_amd/lib/base) against HEAD's on the trees in TREES
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06; mkdir -p $OUT
export TMPDIR=/tmp
TAG=${TAG:-ab}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${K:-uts}" > $OUT/${TAG}_tests.log 2>&1 || { tail -30 $OUT/${TAG}_tests.log; exit 1; }
tail -2 $OUT/${TAG}_tests.log
for t in ${TREES:-T3L}; do
  timeout -k 10 400 python -u scripts/ab_libs_t3l.py $t hclib_amd/lib/base/libhclib_amd.so hclib_amd/lib/libhclib_amd.so >> $OUT/${TAG}.log 2>&1 || exit $?
done
cat $OUT/${TAG}.log
