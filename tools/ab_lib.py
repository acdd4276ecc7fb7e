"""Run a tool script against another build of libmjx.so (an experiment or
diagnostic variant made by _build.build_variant, e.g. ab/libmjx_<tag>.so):

    python tools/ab_lib.py ab/libmjx_nocompute.so tools/hpr_q_time.py
    python tools/ab_lib.py --build nocompute -DMJX_HPR_NOCOMPUTE mjx_hpr_f32.hip   (CPU: make the variant)

The variant's build id carries its flags, so it is opened unverified here and
never by the product loader."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if sys.argv[1] == "--build":
    import mjx
    tag, flags, units = sys.argv[2], [a for a in sys.argv[3:] if a.startswith("-")], \
        [a for a in sys.argv[3:] if not a.startswith("-")]
    out = os.path.join(ROOT, "ab", f"libmjx_{tag}.so")
    mjx._lib._build.build_variant(out, flags, units)
    print(out)
    sys.exit(0)

import mjx  # noqa: E402
path, script = os.path.abspath(sys.argv[1]), sys.argv[2]
mjx._lib._LIB = mjx._lib.open_library(path, verify=False)
print(f"[ab_lib] {os.path.relpath(path, ROOT)}", flush=True)
sys.argv = [script] + sys.argv[3:]
runpy.run_path(script, run_name="__main__")
