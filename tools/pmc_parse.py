#!/usr/bin/env python3
"""Turn rocprofv3 --pmc CSVs (FETCH_SIZE pass, WRITE_SIZE pass) into
profiles/pmc_traffic.json: measured HBM bytes per launch of each kernel.

Correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE/WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reads half the bytes of a wide (16 B/lane) coalesced
stream, so the read side is doubled.  The calibration copy of tools/pmc_run.py
(known byte count) is reported beside it so the factor can be checked on the
same box: calib.read_factor = known read bytes / (FETCH_SIZE*1024).

usage: pmc_parse.py FETCH_DIR WRITE_DIR CALIB_BYTES OUT_JSON
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(dirname, counter):
    """kernel name -> list of counter values (one per dispatch)."""
    vals = defaultdict(list)
    files = glob.glob(os.path.join(dirname, "**", "*counter_collection*.csv"), recursive=True)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def main():
    fdir, wdir, calib_bytes, out = sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4]
    fetch = load(fdir, "FETCH_SIZE")
    write = load(wdir, "WRITE_SIZE")
    res = {"_method": ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                       "tools/pmc_run.py; bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 per dispatch "
                       "(gfx950 FETCH_SIZE half-count correction), averaged over dispatches")}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fk = sum(f) / len(f) if f else 0.0
        wk = sum(w) / len(w) if w else 0.0
        entry = {"dispatches": max(len(f), len(w)), "fetch_kib": fk, "write_kib": wk,
                 "read_bytes_corrected": 2 * fk * 1024, "write_bytes": wk * 1024,
                 "bytes_per_launch": 2 * fk * 1024 + wk * 1024}
        res[short(k)] = entry
    # calibration: the copy dispatch whose write is closest to the known count
    best = None
    for k in set(fetch) & set(write):
        if "copy" not in k.lower() or len(fetch[k]) != len(write[k]):
            continue
        for fk, wk in zip(fetch[k], write[k]):
            err = abs(wk * 1024 - calib_bytes)
            if best is None or err < best[0]:
                best = (err, k, fk, wk)
    if best is not None:
        _, ck, fk, wk = best
        res["_calibration"] = {
            "kernel": short(ck), "known_read_bytes": calib_bytes, "known_write_bytes": calib_bytes,
            "fetch_bytes_raw": fk * 1024, "write_bytes_raw": wk * 1024,
            "read_factor": calib_bytes / max(1.0, fk * 1024),
            "write_factor": calib_bytes / max(1.0, wk * 1024),
        }
    # bench.py key: the fused-count sweep and the plain sweep of the d=4 rollout
    # (the SA section's d=3 level sweeps are other launches)
    sweeps = [v for k, v in res.items() if "k_sweep_ell_rp<4," in k]
    if sweeps:
        tot = sum(v["bytes_per_launch"] * v["dispatches"] for v in sweeps)
        cnt = sum(v["dispatches"] for v in sweeps)
        res["k_sweep_ell_rp"] = {"bytes_per_launch": tot / cnt, "dispatches": cnt}
    # HPR (C3) and binned C5 kernels: one entry per kernel family (the
    # unqualified name without template arguments; k_bin_apply covers _flat)
    def base(k):
        return k.split("<")[0].split("::")[-1].strip()
    fams = {"k_hpr_update_pipe": lambda b: b == "k_hpr_update_pipe",
            "k_hpr_update": lambda b: b == "k_hpr_update",
            "k_hpr_edge_z": lambda b: b == "k_hpr_edge_z",
            "k_hpr_update_q3": lambda b: b == "k_hpr_update_q3",
            "k_hpr_edge_z_q": lambda b: b == "k_hpr_edge_z_q",
            "k_sweep_cls_rp": lambda b: b.startswith("k_sweep_cls"),
            "k_hpr_node_marg": lambda b: b == "k_hpr_node_marg",
            "k_bin_msg": lambda b: b == "k_bin_msg",
            "k_bin_apply": lambda b: b.startswith("k_bin_apply"),
            "k_sa_spec": lambda b: b == "k_sa_spec"}
    entries = {k: v for k, v in res.items() if isinstance(v, dict) and "fetch_kib" in v}
    for fam, match in fams.items():
        ks = [v for k, v in entries.items() if match(base(k))]
        if ks:
            tot = sum(v["bytes_per_launch"] * v["dispatches"] for v in ks)
            cnt = sum(v["dispatches"] for v in ks)
            res[fam] = {"bytes_per_launch": tot / cnt, "dispatches": cnt}
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
