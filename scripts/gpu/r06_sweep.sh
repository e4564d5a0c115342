#!/bin/bash
# round 6: an interleaved knob sweep (scripts/sweep_env.py) on one tree:
#   TREE=T1 ROUNDS=3 REPS=5 bash scripts/gpu/r06_sweep.sh 'K=V' ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06; mkdir -p $OUT
export TMPDIR=/tmp
TAG=${TAG:-sweep_$TREE}
HX_REPS=${REPS:-5} timeout -k 10 ${LIMIT:-500} python -u scripts/sweep_env.py $TREE ${ROUNDS:-3} "$@" > $OUT/$TAG.log 2>&1
rc=$?
grep -v "^round" $OUT/$TAG.log
exit $rc
