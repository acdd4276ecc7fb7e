"""Where a k_sa_spec launch's time goes across its waves (configs[1]: d=3,
N=1e6, p=2, c=1, R=4096; Philox stream, so one step launch per call).  Run
against the diagnostic variant (per-wave start / end real time, batch count
and hardware placement):

    python tools/ab_lib.py --build wavet -DMJX_SA_PROF tools/variants/spec_wavetime.patch mjx_sa.hip   (CPU)
    python tools/ab_lib.py ab/libmjx_wavet.so tools/sa_wave_time.py                                   (GPU)
"""
import collections
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import mjx  # noqa: E402

raw = mjx._lib._LIB
n, d, p, c, R = 1_000_000, 3, 2, 1, 4096
adj = mjx.random_regular_graph(d, n, seed=7)
sa = mjx.SAReplicas(adj, p, c, np.arange(R), mode="lightcone", rng=os.environ.get("SA_RNG", "philox"), tape=8192)
sa.steps(10000)
torch.cuda.synchronize()
nw = (R // 64) * 8
for K in [int(x) for x in os.environ.get("SA_KS", "250,2000,4000").split(",")]:
    for rep in range(2):
        sa.steps(K)
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (4 * nw))()
        raw.mjx_sa_wave_read(buf, 4 * nw)
        a = np.frombuffer(buf, dtype=np.uint64).reshape(nw, 4).astype(np.int64)
        t0, t1, nb, hw = a[:, 0], a[:, 1], a[:, 2], a[:, 3]
        base = t0.min()
        st = (t0 - base) / 100.0          # 100 MHz -> us
        en = (t1 - base) / 100.0
        dur = en - st
        xcc = (hw >> 32) & 0xF
        hid = hw & 0xFFFFFFFF
        simd, cu, sh, se = (hid >> 4) & 3, (hid >> 8) & 15, (hid >> 12) & 1, (hid >> 13) & 7
        cu_key = xcc * 1000 + se * 100 + sh * 16 + cu
        occ = collections.Counter(cu_key.tolist())
        per_cu = np.array([occ[k] for k in cu_key.tolist()])
        simd_key = cu_key * 4 + simd
        socc = collections.Counter(simd_key.tolist())
        per_simd = np.array([socc[k] for k in simd_key.tolist()])
        print(f"K={K} rep {rep}: launch span {en.max():.1f} us; start spread {st.max():.1f} us; "
              f"wave dur min/med/p90/max {dur.min():.1f}/{np.median(dur):.1f}/{np.percentile(dur, 90):.1f}/{dur.max():.1f}; "
              f"batches min/med/max {nb.min()}/{int(np.median(nb))}/{nb.max()}; "
              f"CUs used {len(occ)}, waves per CU hist {sorted(collections.Counter(occ.values()).items())}, "
              f"waves per SIMD hist {sorted(collections.Counter(socc.values()).items())}", flush=True)
        for w in sorted(set(per_cu.tolist())):
            sel = per_cu == w
            print(f"    waves sharing a CU = {w}: {sel.sum()} waves, dur med {np.median(dur[sel]):.1f} max {dur[sel].max():.1f}, "
                  f"us/batch med {np.median(dur[sel] / nb[sel]):.3f}", flush=True)
        for w in sorted(set(per_simd.tolist())):
            sel = per_simd == w
            print(f"    waves sharing a SIMD = {w}: {sel.sum()} waves, dur med {np.median(dur[sel]):.1f} max {dur[sel].max():.1f}",
                  flush=True)
        for x in range(8):
            sel = xcc == x
            if sel.any():
                print(f"    xcc {x}: {sel.sum()} waves, dur med {np.median(dur[sel]):.1f} max {dur[sel].max():.1f}", flush=True)
        slow = np.argsort(-dur)[:6]
        print("    slowest waves: " + ", ".join(f"blk {b} dur {dur[b]:.1f} nb {nb[b]} cu-occ {per_cu[b]} simd-occ {per_simd[b]}"
                                          for b in slow), flush=True)
