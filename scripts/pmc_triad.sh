#!/bin/bash
# HBM traffic of the triad kernel from rocprofv3 PMC counters, one counter
# group per pass (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/fetch -o f -- python3 scripts/triad_pmc_run.py > gpurun_out/pmc/fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/write -o w -- python3 scripts/triad_pmc_run.py > gpurun_out/pmc/write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d gpurun_out/pmc/req -o r -- python3 scripts/triad_pmc_run.py > gpurun_out/pmc/req.log 2>&1 && echo pmc ok
