"""Check an MCMC_p3_d4.npz written by tools/sa_script_run.py on the CPU: every
replica's final configuration, rolled out p + c - 1 = 3 majority steps on its
own graph by the numpy oracle (code/SA_RRG.py:18-26 restated), reaches
m(s_endstate(s)) = 1 (the script's stop, code/SA_RRG.py:84), mag_reached is m(s)
(code/SA_RRG.py:86), and every graph is 4-regular and simple.

    python tools/sa_script_check.py profiles/r04_MCMC_p3_d4.npz
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from oracle import majority as orc  # noqa: E402

with np.load(sys.argv[1], allow_pickle=False) as z:
    z = {k: z[k] for k in z.files}
ok = True
for k in range(len(z["num_steps"])):
    g, s = z["graphs"][k], z["conf"][k].astype(np.int64)
    n = len(s)
    end = np.asarray(orc.s_endstate(g, s, 3, 1)).reshape(-1)
    simple = all(len(set(row)) == 4 and i not in row for i, row in enumerate(g.tolist()))
    deg = np.bincount(g.reshape(-1), minlength=n)
    good = end.mean() == 1.0 and abs(s.mean() - z["mag_reached"][k]) < 1e-12 and simple and (deg == 4).all()
    ok &= bool(good)
    print(f"replica {k}: num_steps {int(z['num_steps'][k])}, mag_reached {z['mag_reached'][k]:.4f} = m(s) "
          f"{s.mean():.4f}, m(s_endstate) {end.mean():.4f}, 4-regular simple graph {simple and (deg == 4).all()}")
print("all replicas at consensus" if ok else "CHECK FAILED")
sys.exit(0 if ok else 1)
