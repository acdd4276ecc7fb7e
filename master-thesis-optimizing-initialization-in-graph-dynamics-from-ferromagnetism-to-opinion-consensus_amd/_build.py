"""Build libmjx.so (hand-written HIP for gfx950) in-tree with hipcc.

Each translation unit is compiled separately because the simulated-annealing
unit needs ``-ffp-contract=off`` (delta_H must round each operation as numpy
does, code/SA_RRG.py:37) while the dynamics unit does not care.
"""
import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
INCLUDE = os.path.normpath(os.path.join(PKG_DIR, "..", "include"))
LIB = os.path.join(PKG_DIR, "libmjx.so")
ARCH = "gfx950"

# (source, extra flags)
UNITS = [
    ("mjx_dynamics.hip", []),
    ("mjx_sa.hip", ["-ffp-contract=off"]),
    ("mjx_hpr.hip", []),
    ("mjx_hpr_f32.hip", []),
    ("mjx_hpr_f64.hip", []),
    ("mjx_hpr_er.hip", []),
    ("mjx_bdcm.hip", ["-ffp-contract=off"]),
    ("mjx_graph.hip", []),
]


def _hipcc():
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: libmjx.so cannot be built")


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    deps.append(os.path.join(INCLUDE, "mjx.h"))
    deps.append(os.path.abspath(__file__))
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


def build(force=False, verbose=True):
    """Compile every HIP unit for gfx950 and link libmjx.so next to this file."""
    if not force and not _stale():
        return LIB
    hipcc = _hipcc()
    objdir = os.path.join(PKG_DIR, "build")
    os.makedirs(objdir, exist_ok=True)
    base = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
            "-Wno-unused-function", "-I", INCLUDE] + os.environ.get("MJX_EXTRA_CFLAGS", "").split()
    objs, cmds = [], []
    # a unit is recompiled when its object is older than its source, any csrc
    # header, include/mjx.h or this script (or always, with force)
    hdrs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hdrs += [os.path.join(INCLUDE, "mjx.h"), os.path.abspath(__file__)]
    newest_hdr = max(os.path.getmtime(p) for p in hdrs if os.path.exists(p))
    for src, extra in UNITS:
        obj = os.path.join(objdir, src.replace(".hip", ".o"))
        srcp = os.path.join(CSRC, src)
        objs.append(obj)
        if (not force and os.path.exists(obj)
                and os.path.getmtime(obj) > max(os.path.getmtime(srcp), newest_hdr)):
            continue
        cmds.append(base + extra + ["-c", srcp, "-o", obj])
    # translation units compile in parallel (the HPR instantiation units dominate)
    from concurrent.futures import ThreadPoolExecutor
    jobs = max(1, min(len(cmds), os.cpu_count() or 1, 8))

    def run(cmd):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)

    with ThreadPoolExecutor(max(1, min(jobs, len(cmds)))) as ex:
        list(ex.map(run, cmds))
    tmp = LIB + ".tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
