"""Time C5 binned-sweep phase-2 variants (env MJX_BIN_BF, a bit set of
k_bin_apply_flat experiments) on one GPU at N=1e9, d=6; exact variants are
checked against variant 0."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mjx  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 6
exps = sys.argv[3].split(",") if len(sys.argv) > 3 else ["0", "1"]
exact = {"0", "1"}
t0 = time.time()
sh = mjx.ShardedRRG(d, n, seed=0, mode="binned")
sh.drop_adjacency()
torch.cuda.synchronize()
print(f"setup {time.time() - t0:.2f}s", flush=True)
s = torch.randint(-2 ** 62, 2 ** 62, (sh.range.words_padded,), dtype=torch.int64, device="cuda")
out = torch.empty_like(s)
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
ref = None
for e in exps:
    os.environ["MJX_BIN_BF"] = e
    for _ in range(2):
        sh.plan.sweep(s, out, cnt)
    torch.cuda.synchronize()
    if e == "0":
        ref = out.clone()
    elif e in exact and ref is not None:
        assert torch.equal(out, ref), f"variant {e} differs"
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        sh.plan.sweep(s, out, cnt)
    e1.record()
    torch.cuda.synchronize()
    print(f"EXP={e}: {e0.elapsed_time(e1) / 5:.3f} ms/sweep", flush=True)
