"""Does a locality relabelling of the graph shrink a light-cone SA ball's cache lines?

VERDICT r02 item 6 proposed relabelling the RRG in BFS / Cuthill-McKee order so that
the radius-2 ball a speculative SA proposal reads (i, its d neighbours, their d(d-1)
other neighbours: 10 nodes at d=3) spans fewer 128-B lines of the cone / record layout.
This counts, for random proposals on a random 3-regular graph of configs[1]'s size,
the distinct 128-B lines holding the ball's per-(node, word column) records, under the
identity labelling, BFS order and reverse Cuthill-McKee order (scipy), for the record
layout (64-B records, 2 per line) and the cone layout (32-B level sectors, 4 per line).

Host-only (numpy/scipy); prints one line per (order, layout).  Round 3 result:
identity 10.0 / 10.0 lines, BFS 9.22 / 8.84, RCM 9.21 / 8.82 -- an expander has no
locality to recover (most nodes sit in the last BFS layers, whose neighbours are
already labelled), far from the 1.5x the item asked for, so the relabelling was not
built.
"""
import numpy as np
import scipy.sparse as sp
import scipy.sparse.csgraph as cg

n, d, samples = 1_000_000, 3, 20000
rng = np.random.default_rng(0)
stubs = rng.permutation(n * d)                       # configuration model (estimate only)
a, b = stubs[0::2] // d, stubs[1::2] // d
A = sp.coo_matrix((np.ones(a.size), (a, b)), shape=(n, n))
A = (A + A.T).tocsr()
A.data[:] = 1
idx, ip = A.indices, A.indptr
ii = rng.integers(0, n, samples)
balls = []
for i in ii:
    l1 = idx[ip[i]:ip[i + 1]]
    l2 = np.concatenate([idx[ip[j]:ip[j + 1]] for j in l1])
    balls.append(np.unique(np.concatenate([[i], l1, l2])))


def lines(perm, rec):
    return np.mean([np.unique(perm[bl] * rec // 128).size for bl in balls])


def as_perm(order):
    perm = np.empty(n, np.int64)
    perm[order] = np.arange(order.size)
    return perm


orders = {
    "identity": np.arange(n),
    "bfs": as_perm(cg.breadth_first_order(A, 0, directed=False, return_predecessors=False)),
    "rcm": as_perm(cg.reverse_cuthill_mckee(A, symmetric_mode=True)),
}
print(f"radius-2 balls at d={d}, n={n}: mean {np.mean([bl.size for bl in balls]):.2f} nodes")
for name, perm in orders.items():
    print(f"{name:9s} record layout (64 B): {lines(perm, 64):.2f} lines   cone layout (32 B): {lines(perm, 32):.2f} lines")
