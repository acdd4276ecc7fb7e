#!/bin/bash
# PMC passes (one counter group per run) over the C5 binned sweep (tools/giant_time.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=gpurun_out/binpmc
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_SALU SQ_WAIT_INST_LDS" \
           "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCC_BUSY_avr" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $grp -d "$R/$OUT/p$i" -o run \
      --output-format csv -- python3 "$R/tools/giant_time.py" 1e9 6 3 ) > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed $?"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob
from collections import defaultdict
acc = defaultdict(list)
for f in glob.glob("gpurun_out/binpmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_bin_msg" in k or "k_bin_apply" in k:
            acc[("msg" if "k_bin_msg" in k else "apply", r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(k, c, sum(v) / len(v))
PY
