"""C5 binned sweep on one GPU (configs[4] single-GPU form): one d-regular graph
of n nodes on the device, its binned plan, HIP-event time per sweep (the
phase kernels k_bin_msg / k_bin_apply_flat show up in a kernel trace).

    python tools/giant_time.py [n=1e9] [d=6] [sweeps=5]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mjx  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 6
K = int(sys.argv[3]) if len(sys.argv) > 3 else 5
t0 = time.time()
sh = mjx.ShardedRRG(d, n, seed=0, mode="binned")
sh.drop_adjacency()
torch.cuda.synchronize()
print(f"setup {time.time() - t0:.2f}s", flush=True)
s = torch.randint(-2 ** 62, 2 ** 62, (sh.range.words_padded,), dtype=torch.int64, device="cuda")
out = torch.empty_like(s)
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
for _ in range(2):
    sh.plan.sweep(s, out, cnt)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(K):
    sh.plan.sweep(s, out, cnt)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / K
print(f"EXP n={n} d={d}: {ms:.3f} ms/sweep, {n / ms * 1e3:.3g} node-updates/s", flush=True)
