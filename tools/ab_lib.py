"""Run a tool script against another build of libmjx.so (an experiment or
diagnostic variant made by _build.build_variant, e.g. ab/libmjx_<tag>.so):

    python tools/ab_lib.py ab/libmjx_nocompute.so tools/hpr_q_time.py
    python tools/ab_lib.py --build nocompute tools/variants/hpr_nocompute.patch mjx_hpr_f32.hip   (CPU)
    python tools/ab_lib.py --build saprof -DMJX_SA_PROF mjx_sa_lds.hip                          (CPU)

Arguments of --build: the tag, then -D/-f flags, *.patch files (unified diffs
against csrc/, applied to a copy: timing builds with wrong results, e.g.
tools/variants/spec_nohash.patch, live only there) and the units to rebuild.
The variant's build id is not a source hash, so it is opened unverified here
and refused by the product loader.  --build first brings the product build up
to date with the working tree (the variant links its other units' objects):
an experiment edited into csrc/ and reverted afterwards needs
__graft_entry__.build() again, or the in-tree libmjx.so no longer matches the
sources and the product loader refuses it."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if sys.argv[1] == "--build":
    import mjx
    args = sys.argv[3:]
    tag = sys.argv[2]
    flags = [a for a in args if a.startswith("-")]
    patches = [a for a in args if a.endswith(".patch")]
    units = [a for a in args if not a.startswith("-") and not a.endswith(".patch")]
    out = os.path.join(ROOT, "ab", f"libmjx_{tag}.so")
    mjx._lib._build.build_variant(out, flags, units, patches=patches)
    print(out)
    sys.exit(0)

import mjx  # noqa: E402
path, script = os.path.abspath(sys.argv[1]), sys.argv[2]
mjx._lib._LIB = mjx._lib.open_library(path, verify=False)
print(f"[ab_lib] {os.path.relpath(path, ROOT)} (build id {mjx._lib._LIB.mjx_build_id().decode()})", flush=True)
sys.argv = [script] + sys.argv[3:]
runpy.run_path(script, run_name="__main__")
