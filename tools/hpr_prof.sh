#!/bin/bash
# HPR (C3) kernel trace + PMC passes on one GPU box: kernel stats, then one
# rocprofv3 --pmc pass per counter group (each its own run, killed at 90 s).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=gpurun_out/hprprof
mkdir -p $OUT
export PYTHONUNBUFFERED=1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$R/$OUT/trace" -o run \
    --output-format csv -- python3 "$R/tools/hpr_time.py" ) > $OUT/trace.log 2>&1 || { echo "trace failed $?"; exit 1; }
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  ( cd /tmp && export TMPDIR=/tmp && ONLY_F32=1 timeout -s KILL 90 rocprofv3 --pmc $grp -d "$R/$OUT/pmc$i" -o run \
      --output-format csv -- python3 "$R/tools/hpr_time.py" ) > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed $?"; exit 1; }
done
echo done
