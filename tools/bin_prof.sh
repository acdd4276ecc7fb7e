#!/bin/bash
# C5 phase-2 variants: timing, kernel trace, LDS/wait PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=gpurun_out/binprof
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 200 python3 tools/bin_exp.py 1e9 6 "${EXPS:-0,2,1,3,4,5}" > $OUT/time.log 2>&1 || { echo "time failed $?"; exit 1; }
cat $OUT/time.log
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/$OUT/trace" -o run \
    --output-format csv -- python3 "$R/tools/bin_exp.py" 1e9 6 "${EXPS:-0,2,1,3,4,5}" ) > $OUT/trace.log 2>&1 || { echo "trace failed $?"; exit 1; }
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $grp -d "$R/$OUT/pmc$i" -o run \
      --output-format csv -- python3 "$R/tools/bin_exp.py" 1e9 6 0 ) > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed $?"; exit 1; }
done
echo done
