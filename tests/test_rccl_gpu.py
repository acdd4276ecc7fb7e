"""The giant-graph exchange (configs[4]) through RCCL on the GPU: a world-1
"nccl" (= RCCL) process group on one MI355X runs exactly the in-place
all_gather_into_tensor / all_reduce calls of the 8-GPU run (piece g's
all-gather on RCCL's stream while piece g+1 is swept), and the rollout equals
the one without collectives and the C oracle on sampled rows.  The multi-rank
exchange itself is covered over gloo (tests/test_partition.py); 8-GPU runs are
the driver's."""
import socket

import numpy as np
import pytest
import torch

from oracle import fast

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


@pytest.mark.parametrize("mode,pieces", [("gather", 2), ("binned", 2), ("gather", 3)])
def test_rccl_exchange_world1(mjx_mod, mode, pieces):
    import torch.distributed as dist
    n, d, steps = 300_000, 6, 3
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", torch.cuda.current_device()))
    try:
        assert dist.get_backend() == "nccl"
        rng = np.random.default_rng(4)
        s = rng.choice(np.array([-1, 1], dtype=np.int8), size=n)
        got = mjx_mod.ShardedRRG(d, n, seed=9, mode=mode, pieces=pieces, collective=True)
        assert got.collective and got.range.npieces == pieces
        got.set_state(s)
        tot = got.rollout(steps)
        ref = mjx_mod.ShardedRRG(d, n, seed=9, mode=mode, pieces=pieces)
        ref.set_state(s)
        assert tot == ref.rollout(steps)
        assert np.array_equal(got.state(), ref.state())
    finally:
        dist.destroy_process_group()
    adj = mjx_mod.random_regular_rows_device(d, n, 9, 0, n).cpu().numpy()
    o = fast.s_endstate(adj, s, steps, 1)          # p + c - 1 = steps
    assert tot == int(o.sum())
