"""Time the C5 binned sweep phases for tuning knobs (env MJX_BIN_APPLY_U) on
one GPU: one d-regular graph, one plan, HIP-event timing per variant."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mjx  # noqa: E402

if os.environ.get("MJX_LIB_OVERRIDE"):   # experiments: time another build of libmjx.so
    mjx._lib._build.LIB = os.environ["MJX_LIB_OVERRIDE"]

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 6
t0 = time.time()
sh = mjx.ShardedRRG(d, n, seed=0, mode="binned")
sh.drop_adjacency()
torch.cuda.synchronize()
print(f"setup {time.time() - t0:.2f}s", flush=True)
s = torch.randint(-2 ** 62, 2 ** 62, (sh.range.words_padded,), dtype=torch.int64, device="cuda")
out = torch.empty_like(s)
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
ref = None
for u in sys.argv[3].split(",") if len(sys.argv) > 3 else ["1", "2", "4"]:
    os.environ["MJX_BIN_APPLY_U"] = u
    for _ in range(2):
        sh.plan.sweep(s, out, cnt)
    torch.cuda.synchronize()
    if ref is None:
        ref = out.clone()
    if not os.environ.get("MJX_LIB_OVERRIDE"):
        assert torch.equal(out, ref), f"variant U={u} differs"
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        sh.plan.sweep(s, out, cnt)
    e1.record()
    torch.cuda.synchronize()
    print(f"U={u}: {e0.elapsed_time(e1) / 5:.3f} ms/sweep", flush=True)
