#!/bin/bash
# Kernel trace of configs[1]'s rec layout (tools/sa_scale.py, R=4096): do the
# side-stream MT tapes overlap the speculative step kernels?
set -u
R="$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
( cd /tmp && export TMPDIR=/tmp && SA_RS=4096 SA_K=2000 SA_LAYOUTS=rec timeout -k 10 300 rocprofv3 --kernel-trace \
    -d "$R/$OUT/c2trace" -o run --output-format csv -- python3 "$R/tools/sa_scale.py" ) > $OUT/c2trace.log 2>&1
