"""Per-device library state: the CU count, occupancy and
dynamic-LDS opt-ins are memoised per device id (mjx_dynamics.hip DevMemo), so
launches after a hipSetDevice round trip run with the current device's
settings and give the same results."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_hpr_dp_after_set_device_round_trip(mjx_mod):
    n, d, p, c = 2000, 4, 2, 2
    plan = mjx_mod.HPRPlan(mjx_mod.random_regular_edges(d, n, seed=5), n, d)
    g = torch.Generator(device="cuda").manual_seed(1)
    chi = torch.rand((2 * plan.E, 4 ** (p + c)), dtype=torch.float32, device="cuda", generator=g)
    chi /= chi.sum(1, keepdim=True)
    b = torch.rand((n, 2), dtype=torch.float32, device="cuda", generator=g)
    b /= b.sum(1, keepdim=True)
    first = mjx_mod.HPr_dp(chi, b, plan, p, c, 1, 25 * n, 0.4).clone()
    dev = torch.cuda.current_device()
    for k in range(torch.cuda.device_count()):      # hipSetDevice to every device and back
        torch.cuda.set_device(k)
    torch.cuda.set_device(dev)
    second = mjx_mod.HPr_dp(chi, b, plan, p, c, 1, 25 * n, 0.4)
    assert torch.equal(first, second)
    assert np.allclose(first.sum(1).cpu().numpy(), 1.0, atol=1e-5)


def test_persistent_grid_sized_by_the_device(mjx_mod):
    """The persistent sweeps size their grid from the device's CU count (the
    rollout of a constant state is that state, whatever the grid)."""
    adj = mjx_mod.random_regular_graph(4, 50_000, seed=2)
    s = torch.full((50_000 * 64,), -1, dtype=torch.int64, device="cuda")
    out = mjx_mod.rollout(mjx_mod.Graph.ell(adj), s, 2, words=64)
    assert torch.equal(out, s)
