#!/bin/bash
# Round-2 profiles at HEAD on one GPU box:
#  1. rocprofv3 --kernel-trace --stats of a short bench.py run (no CPU legs),
#  2. two --pmc passes (FETCH_SIZE, WRITE_SIZE), each its own run, over
#     tools/pmc_run.py (C2 sweep, C3 HPR iteration, C5 binned sweeps),
#     parsed into gpurun_out/prof/pmc_traffic.json by tools/pmc_parse.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=gpurun_out/prof
mkdir -p $OUT
export PYTHONUNBUFFERED=1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$OUT/trace" -o run \
    --output-format csv -- python3 "$R/bench.py" --steps 10 --no-cpu-baseline ) > $OUT/trace.log 2>&1 \
    || { echo "trace failed $?"; exit 1; }
echo trace ok
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $grp -d "$R/$OUT/pmc_$grp" -o run \
      --output-format csv -- python3 "$R/tools/pmc_run.py" ) > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $grp failed $?"; exit 1; }
  echo "pmc $grp ok"
done
python3 tools/pmc_parse.py $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE $((1024*1024*1024)) $OUT/pmc_traffic.json > $OUT/parse.log
echo done
