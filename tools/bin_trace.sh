#!/bin/bash
# kernel trace of the C5 binned sweep under knob settings (env lists), one process each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=gpurun_out/bintrace
mkdir -p $OUT
for sp in ${SPLITS:-4}; do for uc1 in ${UC1S:-4}; do for uc2 in ${UC2S:-2}; do
  tag=s${sp}_a${uc1}_b${uc2}
  ( cd /tmp && export TMPDIR=/tmp && MJX_BIN_SPLIT=$sp MJX_BIN_UC1=$uc1 MJX_BIN_UC2=$uc2 timeout -k 10 100 rocprofv3 --kernel-trace -d "$R/$OUT/$tag" -o run \
      --output-format csv -- python3 "$R/tools/bin_exp.py" 1e9 6 0 ) > $OUT/$tag.log 2>&1 || { echo "trace $tag failed"; exit 1; }
  python3 - "$OUT/$tag" "$tag" <<'PY'
import csv, glob, sys
from collections import defaultdict
d = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_bin_msg" in k or "k_bin_apply" in k:
            d["msg" if "k_bin_msg" in k else "apply"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(sys.argv[2], {k: round(sorted(v)[len(v) // 2], 1) for k, v in d.items()})
PY
done; done; done
