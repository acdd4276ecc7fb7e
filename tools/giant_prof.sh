#!/bin/bash
# Giant-graph (C5) bench leg alone, then the same under rocprofv3 --kernel-trace --stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=gpurun_out
mkdir -p $OUT
ARGS="--no-cpu-baseline --no-sa --no-er --no-bdcm --steps 3 ${GIANT_ARGS:-}"
timeout -k 10 300 python -u bench.py $ARGS > $OUT/bench_giant.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$OUT/prof" -o run --output-format csv -- \
    python3 "$R/bench.py" $ARGS > "$R/$OUT/prof.log" 2>&1
