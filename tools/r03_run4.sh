#!/bin/bash
# round 3, GPU session 4: HPR parity after the no-SLP build, the HPR timing, the bench and its kernel trace
set -o pipefail
O=gpurun_out; mkdir -p $O
PYTEST_PATHS="tests/test_hpr_gpu.py tests/test_hpr_q_gpu.py tests/test_hpr_er_gpu.py tests/test_drop_in.py" \
  STEPS="tests" bash tools/gpu_check.sh || exit $?
ONLY_F32=1 timeout -k 10 120 python -u tools/hpr_time.py > $O/hpr_time.log 2>&1 || exit $?
PROF_ARGS="--no-consensus" STEPS="bench prof" bash tools/gpu_check.sh || exit $?
