#!/bin/bash
# round 3, GPU session 9: branch-free hash probes in the speculative SA kernel (.wip2): phase timers + parity
set -o pipefail
O=$PWD/gpurun_out; mkdir -p $O
( cd .wip2 && SA_RS=1024,4096,16384 timeout -k 10 300 python -u tools/sa_prof.py ) > $O/C_sa_prof4.log 2>&1 || exit $?
( cd .wip2 && timeout -k 10 600 python -u -m pytest tests/test_sa_gpu.py tests/test_sa_multi_gpu.py -m gpu -x -q \
    --timeout 200 --timeout-method thread ) > $O/C_sa_tests.log 2>&1 || exit $?
