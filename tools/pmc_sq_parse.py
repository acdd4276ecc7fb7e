#!/usr/bin/env python3
"""Summarise the SQ counter pass (tools/gpu_check.sh step `sq`) per kernel:
profiles/rNN_sq_counters.json.

SQ_WAVE_CYCLES, SQ_WAIT_ANY and SQ_ACTIVE_INST_VALU count quad-cycles of
resident waves (MI355X_MICROARCH.md, PMC section), so their ratios are the
fraction of a wave's resident time spent waiting (s_waitcnt / barrier) and
issuing VALU work; GRBM_GUI_ACTIVE / 8 is the dispatch's GPU cycles per XCD.

usage: pmc_sq_parse.py SQ_DIR OUT_JSON
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    sqdir, out = sys.argv[1], sys.argv[2]
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(sqdir, "**", "*counter_collection*.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"].split("(")[0].replace("void ", "").strip()
                vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {"_method": "rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS "
                      "SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE over tools/pmc_run.py "
                      "--no-giant --no-er; per-dispatch means; wait_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES, "
                      "valu_active_frac = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (both quad-cycle counts)"}
    for k, d in sorted(vals.items()):
        m = {c: sum(v) / len(v) for c, v in d.items()}
        e = {"dispatches": max(len(v) for v in d.values()), **{c: m[c] for c in sorted(m)}}
        wc = m.get("SQ_WAVE_CYCLES", 0.0)
        if wc > 0:
            e["wait_frac"] = m.get("SQ_WAIT_ANY", 0.0) / wc
            e["valu_active_frac"] = m.get("SQ_ACTIVE_INST_VALU", 0.0) / wc
        if m.get("SQ_WAVES"):
            e["valu_insts_per_wave"] = m.get("SQ_INSTS_VALU", 0.0) / m["SQ_WAVES"]
        res[k] = e
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(f"{len(res) - 1} kernels -> {out}")


if __name__ == "__main__":
    main()
