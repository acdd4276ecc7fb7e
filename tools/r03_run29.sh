#!/bin/bash
# round 3, GPU session 29: plain-store mark clears, schedule by shuffle in the pair step: parity, step times, phase timers
set -o pipefail
O=$PWD/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sa_gpu.py tests/test_sa_multi_gpu.py -m gpu -x -q --timeout 200 \
    --timeout-method thread > $O/U_sa_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/sa_probe3.py > $O/U_sa_probe3.log 2>&1 || exit $?
( cd .wip3 && timeout -k 10 300 python -u tools/sa_lds_prof.py ) > $O/U_sa_lds_prof.log 2>&1 || exit $?
