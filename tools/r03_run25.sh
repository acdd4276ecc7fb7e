#!/bin/bash
# round 3, GPU session 25: fused HPR node step (marginal + bias refresh + s + packed bits): parity and loop time
set -o pipefail
O=$PWD/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_hpr_q_gpu.py tests/test_hpr_gpu.py tests/test_drop_in.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > $O/Q_hpr_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/hpr_loop_time.py > $O/Q_hpr_loop.log 2>&1 || exit $?
