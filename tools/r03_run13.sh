#!/bin/bash
# round 3, GPU session 13: lane-held LDS SA step (k_sa_lds_fast): parity tests, then step times
set -o pipefail
O=$PWD/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sa_gpu.py tests/test_sa_multi_gpu.py -m gpu -x -v --timeout 200 \
    --timeout-method thread > $O/F_sa_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/sa_probe3.py > $O/F_sa_probe3.log 2>&1 || exit $?
