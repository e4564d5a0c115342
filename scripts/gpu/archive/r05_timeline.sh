#!/bin/bash
# worker timelines on the timeline build (scripts/uts_timeline.py); TREES / OUTF from the env
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
HCLIB_AMD_LIB=hclib_amd/lib/timeline/libhclib_amd.so timeout -k 10 300 python -u scripts/uts_timeline.py gpurun_out/r05/${OUTF:-timeline}.jsonl ${TREES:-T1} > gpurun_out/r05/${OUTF:-timeline}.log 2>&1
rc=$?; tail -5 gpurun_out/r05/${OUTF:-timeline}.log; exit $rc
