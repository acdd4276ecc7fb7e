"""Driver for SQ counter passes over the whole-CU LDS SA kernel alone
(SA_RRG.py's p=3, c=1: d=4, n=1e4, 64 replicas on distinct graphs):

    rocprofv3 --pmc <SQ counters> -d OUT -o run --output-format csv -- python3 tools/sa_wg_pmc.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mjx  # noqa: E402

n, d, R = 10_000, 4, 64
graphs = [mjx.random_regular_graph(d, n, seed=7000 + k) for k in range(R)]
sa = mjx.SAReplicas(graphs, 3, 1, list(range(R)), layout="lds")
for _ in range(4):
    sa.steps(5000)
torch.cuda.synchronize()
print("sa_wg_pmc done", flush=True)
