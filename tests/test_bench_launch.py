"""bench.py's launcher: `--gpus N` without a
torch.distributed.run environment starts N rank processes; the dry-run mode
drives the same path over gloo without a GPU.  `--gpus 1` stays one process."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(argv, env_extra=None, timeout=120):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + argv, capture_output=True, text=True, timeout=timeout,
                          env=env, cwd=ROOT)


def _json_lines(out):
    return [json.loads(x) for x in out.splitlines() if x.strip().startswith("{")]


@pytest.mark.parametrize("n", [2, 3, 8])
def test_gpus_n_starts_n_ranks_and_prints_one_line(n):
    p = _run(["--gpus", str(n), "--dry-run", "--steps", "3", "--warmup", "1"])
    assert p.returncode == 0, p.stderr
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    line = lines[0]
    assert line["n_gpus"] == n and line["ranks"] == n
    pids = line["rank_pids"]
    assert len(pids) == n and len(set(pids)) == n           # n distinct processes
    assert os.getpid() not in pids
    assert line["steps"] == 3 and line["warmup"] == 1


def test_torch_distributed_run_launch_8_ranks():
    """The driver's own N = 8 command line (python -m torch.distributed.run
    --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 ... bench.py --gpus 8),
    dry-run: eight ranks from the launcher's environment, one line from rank 0."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), BENCH, "--gpus", "8", "--dry-run",
                        "--steps", "3", "--warmup", "1"], capture_output=True, text=True, timeout=240, env=env,
                       cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    (line,) = _json_lines(p.stdout)
    assert line["n_gpus"] == 8 and len(set(line["rank_pids"])) == 8


def test_gpus_1_is_one_process():
    p = _run(["--gpus", "1", "--dry-run"])
    assert p.returncode == 0, p.stderr
    (line,) = _json_lines(p.stdout)
    assert line["n_gpus"] == 1 and len(line["rank_pids"]) == 1


def test_world_size_mismatch_fails():
    p = _run(["--gpus", "4", "--dry-run"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE" in p.stderr
    assert not _json_lines(p.stdout)


def test_too_few_gpus_fails_loudly():
    """No GPU in this container: --gpus 2 must refuse instead of reporting n_gpus 1."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("two GPUs visible")
    p = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert p.returncode != 0
    assert "visible" in p.stderr
    assert not _json_lines(p.stdout)


def test_bench_reads_committed_pmc_traffic():
    """The bench line's `traffic` fields come from profiles/pmc_traffic.json:
    the headline sweep's bytes per launch, and the ER step's plain and
    counting sweeps (the counting one now k_sweep_cls_all_rp + the D > 8
    tail), each within a few percent of the algorithmic bytes."""
    sys.path.insert(0, ROOT)
    import bench
    t = bench.rocprof_traffic()
    assert t is not None and abs(t / 3.088e9 - 1) < 0.05        # d=4, N=1e6, R=4096: 3088 B per node
    er = bench.er_sweep_traffic()
    assert er is not None
    assert abs(er["counting_sweep_bytes"] / er["plain_sweep_bytes"] - 1) < 0.05


def test_printed_line_is_compact_and_ends_with_the_summary():
    """the driver keeps only the tail of stdout (~8 KB, the
    record's `tail` 2 KB), so the printed line keeps each leg's numbers, moves
    prose and per-replica arrays to the detail file, and ends with `summary`
    (every config's headline number).  Built here from a committed full bench
    object (round 5's last bench, all legs present)."""
    sys.path.insert(0, ROOT)
    import bench
    line = json.load(open(os.path.join(ROOT, "profiles", "r05_final_b_bench.json")))
    out = {k: (bench.compact(v) if k in bench.LEG_KEYS else v) for k, v in line.items()}
    out["detail_file"] = "gpurun_out/bench_detail.json"
    out["summary"] = bench.summary(line)
    text = json.dumps(out, separators=(",", ":"))
    assert len(text) < 7000
    assert list(out)[-1] == "summary"
    tail = text[-2000:]
    for key in ("c2_mt_props_per_s", "c1_props_per_s", "c4_ms_per_step", "c3_hpr_dp_ms", "c5_ms_per_sweep",
                "c5_setup_s", "sa_global_wall_s"):
        assert f'"{key}":' in tail, key
    assert out["summary"]["c2_mt_props_per_s"] > 1e9
    # the contract's own keys stay whole, cpu_baseline with its sample
    assert out["cpu_baseline"]["sample"] and out["roofline"]["frac"] == line["roofline"]["frac"]
    assert "done_num_steps" not in json.dumps(out["sa_consensus"])
