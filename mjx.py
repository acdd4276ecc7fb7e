"""Import shim: ``import mjx`` loads the package directory
master-thesis-optimizing-initialization-in-graph-dynamics-from-ferromagnetism-to-opinion-consensus_amd/
(whose name is not a Python identifier) under the name ``mjx``."""
import importlib.util as _ilu
import os as _os
import sys as _sys

PKG_DIR = _os.path.join(
    _os.path.dirname(_os.path.abspath(__file__)),
    "master-thesis-optimizing-initialization-in-graph-dynamics-from-ferromagnetism-to-opinion-consensus_amd")

_spec = _ilu.spec_from_file_location("mjx", _os.path.join(PKG_DIR, "__init__.py"),
                                     submodule_search_locations=[PKG_DIR])
_mod = _ilu.module_from_spec(_spec)
_sys.modules["mjx"] = _mod
_spec.loader.exec_module(_mod)

if __name__ == "__main__":
    # python -m mjx sa|hpr|bdcm ...: the reference's experiments with its
    # constants as flags (package module cli.py)
    import importlib as _il
    _il.import_module("mjx.cli").main(_sys.argv[1:])
