"""ORACLE (test infrastructure only): build recipe for the C restatement
oracle/orc_majority.c -> oracle/liborc.so (gcc; called by
__graft_entry__.build()).  The product library never links it."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "orc_majority.c")
LIB = os.path.join(HERE, "liborc.so")


def build(force=False, verbose=True):
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) > os.path.getmtime(SRC):
        return LIB
    # -ffp-contract=off: delta_H rounds every operation like numpy (code/SA_RRG.py:37)
    cmd = ["gcc", "-O2", "-std=gnu99", "-ffp-contract=off", "-fPIC", "-shared", "-o", LIB + ".tmp", SRC, "-lm"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
