"""Per wave and round instruction counts of k_sa_lds_wg<4, 3, 16> from the two
SQ passes of tools/sa_wg_pmc.sh (gpurun_out/sqa.json, sqb.json); rounds per
dispatch from the phase-timer log's proposals per round (argument)."""
import json
import sys

ppr = float(sys.argv[1]) if len(sys.argv) > 1 else 14.0
m = {}
for f in ("gpurun_out/sqa.json", "gpurun_out/sqb.json"):
    for k, v in json.load(open(f)).items():
        if "k_sa_lds_wg<4, 3, 16" in k:
            m.update(v)
waves = m["SQ_WAVES"]
rounds = 5000 / ppr
for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
    print(f"{c}: {m[c] / waves / rounds:.0f} per wave-round")
wc = m["SQ_WAVE_CYCLES"]
for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA",
          "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
    print(f"{c}/WAVE_CYCLES: {m[c] / wc:.3f}")
print(f"LDS bank conflict / idx active: {m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:.3f}")
