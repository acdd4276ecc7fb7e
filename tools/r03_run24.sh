#!/bin/bash
# round 3, GPU session 24: LDS SA at T = 4 (pair / single) against the oracle
set -o pipefail
O=$PWD/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sa_multi_gpu.py -m gpu -x -v --timeout 200 \
    --timeout-method thread -k "lds" > $O/P_sa_t4.log 2>&1 || exit $?
