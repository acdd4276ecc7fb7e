#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/timeout (exit status other
# than 0 = pass or 1 = test failures) ends the script before the next step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export PYTHONUNBUFFERED=1
stop_if_fatal() {  # $1 = status, $2 = step name
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then
    echo "FATAL: step $2 exited with $1; no further GPU steps" | tee -a $OUT/steps.log
    exit "$1"
  fi
  echo "step $2 -> $1" | tee -a $OUT/steps.log
}
STEPS="${STEPS:-tests bench prof}"
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${PYTEST_PATHS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
        ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
      stop_if_fatal $? tests ;;
    py)
      # probe scripts, ";;"-separated: PY="tools/sa_probe3.py --no-cone ;; tools/hpr_q_time.py"
      # (logs py_1.log, py_2.log, ...; PY_LOG=name for a single one)
      k=0
      IFS=$'\n'; for cmd in $(echo "$PY" | sed 's/ *;; */\n/g'); do
        unset IFS
        k=$((k+1))
        log=${PY_LOG:-py_$k}
        timeout -k 10 ${PY_TIMEOUT:-300} python -u $cmd > $OUT/$log.log 2>&1
        stop_if_fatal $? "py $cmd"
      done
      unset IFS ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      stop_if_fatal $? smoke ;;
    bench)
      timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
      stop_if_fatal $? bench ;;
    prof)
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
          -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- \
          python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline ${PROF_ARGS:-${BENCH_ARGS:-}} ) > $OUT/prof.log 2>&1
      stop_if_fatal $? prof ;;
    pmc)
      R="$GRAFT_REPO_ROOT"
      ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE \
          -d "$R/$OUT/pmc_fetch" -o run --output-format csv -- python3 "$R/tools/pmc_run.py" ) > $OUT/pmc_fetch.log 2>&1
      stop_if_fatal $? pmc_fetch
      ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE \
          -d "$R/$OUT/pmc_write" -o run --output-format csv -- python3 "$R/tools/pmc_run.py" ) > $OUT/pmc_write.log 2>&1
      stop_if_fatal $? pmc_write
      python3 tools/pmc_parse.py $OUT/pmc_fetch $OUT/pmc_write $((1024*1024*1024)) $OUT/pmc_traffic.json > $OUT/pmc_parse.log 2>&1
      echo "pmc parse -> $?" | tee -a $OUT/steps.log ;;
    sq)
      # compute-side counters (one SQ pass: 8 SQ + 1 GRBM) over the HPR / SA / sweep workload
      R="$GRAFT_REPO_ROOT"
      ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
          SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
          -d "$R/$OUT/pmc_sq" -o run --output-format csv -- python3 "$R/tools/pmc_run.py" --no-giant --no-er ) > $OUT/pmc_sq.log 2>&1
      stop_if_fatal $? pmc_sq ;;
  esac
done
echo done
