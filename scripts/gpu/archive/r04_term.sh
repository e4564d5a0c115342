#!/bin/bash
# round 4: termination flags in the deque headers, per-XCD hints
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp HCLIB_HIP_SPIN_LIMIT_MS=5000
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "uts or fib or cross_gpu" > gpurun_out/r04/term_tests.log 2>&1 &&
timeout -k 10 200 python -u scripts/uts_probe.py T1 T1L T1XL:7 T1XL T3L fib30 > gpurun_out/r04/term_probe.log 2>&1 &&
timeout -k 10 240 env HCLIB_AMD_LIB=hclib_amd/lib/timeline/libhclib_amd.so python -u scripts/uts_timeline.py gpurun_out/r04/timeline_term.jsonl T1 T1L T1XL:7 > gpurun_out/r04/timeline_term.log 2>&1 &&
timeout -k 10 120 scripts/ubench/ub_valu2.bin > gpurun_out/r04/ub_valu2.log 2>&1 &&
echo ok
