"""The script-shaped fronts (python -m mjx sa|hpr|bdcm): every flag named
after one of the reference's module constants defaults to that constant's
value (code/SA_RRG.py:44-52, code/HPR_pytorch_RRG.py:224-251,
code/ER_BDCM_entropy.ipynb raw lines 456-481).  CPU only: argument parsing.
When the reference tree is present (the build container) its constants are
also read from the files' text (ast of the module-level assignments)."""
import ast
import json
import os

import numpy as np
import pytest

REF = "/root/reference/code"


def _cli(mjx_mod):
    import importlib
    return importlib.import_module("mjx.cli")


def test_defaults_are_the_reference_constants(mjx_mod):
    cli = _cli(mjx_mod)
    ap = cli.build_parser()
    for cmd, table in (("sa", cli.SA_DEFAULTS), ("hpr", cli.HPR_DEFAULTS), ("bdcm", cli.BDCM_DEFAULTS)):
        a = vars(ap.parse_args([cmd]))
        for k, v in table.items():
            assert a[k] == v, (cmd, k, a[k], v)
        assert a["seed"] == 0 and a["gpus"] == 1 and a["replicas"] is None
    assert cli.SA_DEFAULTS == {"n": 10000, "d": 4, "p": 3, "c": 1, "par_a": 1.0005, "par_b": 1.0005, "N_stat": 5}
    a = ap.parse_args(["sa", "--n", "1000", "--p", "1", "--N_stat", "2", "--replicas", "7", "--gpus", "2"])
    assert (a.n, a.p, a.N_stat, a.replicas, a.gpus) == (1000, 1, 2, 7, 2)


def _module_constants(src):
    out = {}
    for node in ast.parse(src).body:
        if isinstance(node, ast.Assign) and len(node.targets) == 1 and isinstance(node.targets[0], ast.Name):
            try:
                out[node.targets[0].id] = ast.literal_eval(node.value)
            except ValueError:
                out[node.targets[0].id] = ast.unparse(node.value)
    return out


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present (GPU box)")
def test_defaults_match_the_reference_files(mjx_mod):
    cli = _cli(mjx_mod)
    sa = _module_constants(open(os.path.join(REF, "SA_RRG.py")).read())
    for k, v in cli.SA_DEFAULTS.items():
        assert sa[k] == v, k
    hpr = _module_constants(open(os.path.join(REF, "HPR_pytorch_RRG.py")).read())
    for k, v in cli.HPR_DEFAULTS.items():
        assert (hpr[k] == "25 * n") if k == "lmbd_in" else (hpr[k] == v), k
    nb = json.load(open(os.path.join(REF, "ER_BDCM_entropy.ipynb")))
    cell = "".join(nb["cells"][0]["source"])
    bd = _module_constants(cell)
    for k, v in cli.BDCM_DEFAULTS.items():
        if k == "deg":
            assert bd[k] == "np.linspace(1, 2, 3)" and np.allclose(np.linspace(1, 2, 3), v)
        else:
            assert bd[k] == v, k


def test_global_stream_refuses_several_gpus(mjx_mod):
    """--stream global is one numpy stream seeded once (code/SA_RRG.py:58-88),
    serial by construction: with --gpus > 1 the front refuses instead of
    quietly running on one device."""
    cli = _cli(mjx_mod)
    a = cli.build_parser().parse_args(["sa", "--n", "100", "--gpus", "2", "--stream", "global"])
    with pytest.raises(SystemExit, match="serial"):
        cli.run_sa(a)
