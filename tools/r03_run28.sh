#!/bin/bash
# round 3, GPU session 28: multi-proposal LDS SA with a vectorised resolution: parity, step times, phase timers
set -o pipefail
O=$PWD/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sa_gpu.py tests/test_sa_multi_gpu.py -m gpu -x -q --timeout 200 \
    --timeout-method thread > $O/T_sa_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/sa_probe3.py > $O/T_sa_probe3.log 2>&1 || exit $?
( cd .wip3 && timeout -k 10 300 python -u tools/sa_lds_prof.py ) > $O/T_sa_lds_prof.log 2>&1 || exit $?
