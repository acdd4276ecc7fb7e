"""Node-range partition of one giant graph on CPU:
world_size 2, 3 and 8 over gloo (8 with the P > 1 default of two pieces per
rank, the world and pieces bench.py --gpus 8 runs the C5 leg at), the
exchange logic of ShardedRRG driven with a reference sweep of each rank's rows
(oracle/majority.py) must reproduce the single-process s_endstate bit for bit.  The HIP local sweep is covered by
tests/test_graph_gpu.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, d, steps, s0, adj, out, pieces):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import mjx
        from oracle import majority as orc
        r = mjx.NodeRange(n, world, rank, pieces)

        def local_sweep(s_in, s_out, counts, g):
            w_lo, w_hi, lo, hi = r.pieces[g]
            spins = mjx.unpack_host(s_in.numpy(), n)
            new = orc.onestep_majority(adj, spins)[lo:hi]
            words = mjx.pack_host(new, w_hi - w_lo)
            s_out[w_lo:w_hi] = torch.from_numpy(words)
            if counts is not None:
                counts += int((new > 0).sum())

        rows = [torch.from_numpy(adj[lo:hi]) for (_, _, lo, hi) in r.pieces]
        sh = mjx.ShardedRRG(d, n, adj_rows=rows, local_sweep=local_sweep, pieces=pieces)
        sh.set_state(s0)
        tot = sh.rollout(steps)
        out[rank] = (sh.state(), tot)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,d,steps,pieces", [(2, 1000, 4, 3, 1), (3, 778, 3, 2, 1), (2, 64, 6, 1, 1),
                                                    (3, 130, 4, 4, 1), (2, 5000, 4, 3, 4), (3, 2000, 3, 2, 3),
                                                    (2, 300, 6, 2, 4), (8, 4000, 6, 2, 2), (8, 1000, 3, 3, 2),
                                                    (8, 640, 4, 2, 2)])
def test_sharded_rollout_matches_oracle(world, n, d, steps, pieces, mjx_mod):
    from oracle import majority as orc
    adj = mjx_mod.random_regular_graph(d, n, seed=world * 100 + n)
    s0 = 2 * np.random.default_rng(n).integers(0, 2, n).astype(np.int64) - 1
    want = orc.s_endstate(adj, s0, steps, 1)
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker, args=(world, port, n, d, steps, s0, adj, out, pieces), nprocs=world, join=True)
        res = dict(out)
    for rank in range(world):
        state, tot = res[rank]
        assert np.array_equal(state, want), rank
        assert tot == int(want.sum())


def test_node_range_covers_every_node(mjx_mod):
    for n in (1, 63, 64, 65, 1000, 10 ** 6 + 3):
        for world in (1, 2, 3, 8):
            rs = [mjx_mod.NodeRange(n, world, r) for r in range(world)]
            assert rs[0].lo == 0 and rs[-1].hi == n
            for a, b in zip(rs, rs[1:]):
                assert a.hi == b.lo
            assert all((r.lo % 64 == 0 or r.lo == n) and (r.hi % 64 == 0 or r.hi == n) for r in rs)
            assert all(r.words_padded == rs[0].chunk * world for r in rs)
    # several pieces per rank: every word owned exactly once, pieces contiguous across ranks
    for n in (1, 65, 1000, 10 ** 6 + 3):
        for world in (1, 2, 3, 8):
            for pieces in (2, 3, 4):
                rs = [mjx_mod.NodeRange(n, world, r, pieces) for r in range(world)]
                owned = np.zeros(rs[0].words_padded, dtype=np.int64)
                for r in rs:
                    for g, (w0, w1, lo, hi) in enumerate(r.pieces):
                        owned[w0:w1] += 1
                        assert lo == min(n, 64 * w0) and hi == min(n, 64 * w1)
                        sl = r.own_words(g)
                        assert sl.start >= r.piece_words(g).start and sl.stop <= r.piece_words(g).stop
                assert np.all(owned[:rs[0].words] == 1) and np.all(owned[rs[0].words:] == 0)
                assert sum(r.rows for r in rs) == n


def test_pack_host_roundtrip(mjx_mod):
    rng = np.random.default_rng(0)
    for n in (1, 63, 64, 65, 1000):
        s = 2 * rng.integers(0, 2, n).astype(np.int64) - 1
        w = mjx_mod.pack_host(s)
        assert w.shape == ((n + 63) // 64,)
        assert np.array_equal(mjx_mod.unpack_host(w, n), s)
        # bit j of word i is node 64 i + j, bit = 1 for +1 (the rp/np layout of include/mjx.h)
        assert ((int(w[0]) >> 0) & 1) == (s[0] > 0)


def test_rrg_pairing_is_an_involution_without_fixed_points(mjx_mod):
    """The device generator's stub pairing (host restatement exported by the
    library): partner(partner(s)) == s, partner(s) != s, for several sizes."""
    lib = mjx_mod.load_library()
    for (n, d, seed) in ((10, 3, 0), (1000, 4, 5), (777, 6, 123456789)):
        ps = np.array([lib.mjx_rrg_partner_host(n, d, seed, s) for s in range(n * d)])
        assert np.array_equal(ps[ps], np.arange(n * d))
        assert not np.any(ps == np.arange(n * d))
    assert lib.mjx_rrg_partner_host(7, 3, 0, 0) == -1          # n*d odd
