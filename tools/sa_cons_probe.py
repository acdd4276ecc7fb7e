"""Progress of a run to consensus (d=4, p=3, c=1) on distinct graphs, printed per chunk."""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402
import mjx  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1000
R = int(sys.argv[2]) if len(sys.argv) > 2 else 2
cap = float(sys.argv[3]) if len(sys.argv) > 3 else 100.0
graphs = [mjx.random_regular_graph(4, n, seed=50 + k) for k in range(R)]
sa = mjx.SAReplicas(graphs, 3, 1, [5 + k for k in range(R)])
print("mode", sa.mode, "layout", sa.layout, flush=True)
t0 = time.perf_counter()
chunk, tot = 1024, 0
while not sa.all_done() and time.perf_counter() - t0 < cap:
    t1 = time.perf_counter()
    sa.steps(chunk)
    torch.cuda.synchronize()
    tot += chunk
    print(f"steps {tot} chunk {chunk}: {1e6 * (time.perf_counter() - t1) / chunk:.2f} us/step, "
          f"t {sa.t.cpu().tolist()[:4]} sum_end {sa.sum_end.cpu().tolist()[:4]} done {sa.done.cpu().tolist()[:4]}",
          flush=True)
    chunk = min(chunk * 2, 65536)
print("wall", time.perf_counter() - t0, flush=True)
res = sa.results()
print("done", int(res["done"].sum()), "of", R, flush=True)
print("num_steps", sorted(res["num_steps"].tolist()), flush=True)
print("mag_reached", res["mag_reached"].tolist(), flush=True)
