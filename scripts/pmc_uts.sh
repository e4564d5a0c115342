#!/bin/bash
# SQ instruction/wait counters of the UTS megakernel, one counter group per pass.
# usage: scripts/pmc_uts.sh TREE GRID OUTDIR   (GRID 0 = default grid)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-T3}; G=${2:-1}; OUT=${3:-gpurun_out/pmcu}
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o p -- python3 scripts/uts_pmc_run.py $T $G > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo pmc ok
