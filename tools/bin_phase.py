"""Phase-level timing of the C5 binned sweep (N=1e9, d=6, one GPU) under the
phase-1 variant knob MJX_BIN_P1 (values from argv, results compared with the
first); run under rocprofv3 --kernel-trace --stats for per-kernel averages."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mjx  # noqa: E402

n = int(float(os.environ.get("BIN_N", "1e9")))
d = int(os.environ.get("BIN_D", "6"))
t0 = time.time()
sh = mjx.ShardedRRG(d, n, seed=0, mode="binned")
sh.drop_adjacency()
torch.cuda.synchronize()
print(f"setup {time.time() - t0:.2f}s", flush=True)
s = torch.randint(-2 ** 62, 2 ** 62, (sh.range.words_padded,), dtype=torch.int64, device="cuda")
out = torch.empty_like(s)
cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
ref = None
for e in (sys.argv[1:] or ["0"]) * 2:
    os.environ["MJX_BIN_P1"] = e
    for _ in range(2):
        sh.plan.sweep(s, out, cnt)
    torch.cuda.synchronize()
    if ref is None:
        ref = out.clone()
    assert torch.equal(out, ref), e
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        sh.plan.sweep(s, out, cnt)
    e1.record()
    torch.cuda.synchronize()
    print(f"EXP={e}: {e0.elapsed_time(e1) / 10:.3f} ms/sweep", flush=True)
