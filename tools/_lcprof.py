import os, sys, time, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, mjx
from mjx import _lib
lib = _lib.load()
n, d, p, c = 1_000_000, 3, 2, 1
adj = mjx.random_regular_graph(d, n, seed=7)
buf = (ctypes.c_ulonglong * 10)()
names = ["l1 batch", "l2a batch", "l2b+finish", "accept math", "flip issue", "flip wait", "rotate", "tree steps", "other cyc", "other steps"]
for cm in (os.environ.get('CMS','0,1').split(',')):
  os.environ['MJX_CONE_CM'] = cm
  for R in (4096, 16384):
      sa = mjx.SAReplicas(adj, p, c, np.arange(R), mode="lightcone")
      sa.steps(2000); torch.cuda.synchronize()
      lib.mjx_lc_prof_read(buf)
      t0 = time.perf_counter(); sa.steps(1000); torch.cuda.synchronize(); el = time.perf_counter() - t0
      lib.mjx_lc_prof_read(buf)
      v = list(buf)
      print(f"cm={cm} R={R}: {1e6*el/1000:.2f} us/step; waves' tree steps {v[7]}, other {v[9]}")
      for k in range(7):
          print(f"   {names[k]:12s} {v[k]/max(v[7],1):8.0f} cyc/step")
      print(f"   other path   {v[8]/max(v[9],1):8.0f} cyc/step")
      del sa
