#!/bin/bash
set -u
R="$GRAFT_REPO_ROOT"
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u tools/sa_scale.py > gpurun_out/sa_scale.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
SA_RS=4096 SA_K=500 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/sa_fetch" -o run --output-format csv -- python3 "$R/tools/sa_scale.py" > $R/gpurun_out/sa_fetch.log 2>&1 || exit $?
SA_RS=4096 SA_K=500 timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$R/gpurun_out/sa_hit" -o run --output-format csv -- python3 "$R/tools/sa_scale.py" > $R/gpurun_out/sa_hit.log 2>&1 || exit $?
