#!/bin/bash
# round 3, GPU session 7: .wip2 = the speculative SA kernel with all first-slot hash probes of a
# lane issued at once (diagnostic build with phase timers): phase timers, then SA parity tests
set -o pipefail
O=$PWD/gpurun_out; mkdir -p $O
( cd .wip2 && SA_RS=1024,4096,16384 timeout -k 10 300 python -u tools/sa_prof.py ) > $O/C_sa_prof2.log 2>&1 || exit $?
( cd .wip2 && timeout -k 10 600 python -u -m pytest tests/test_sa_gpu.py tests/test_sa_multi_gpu.py -m gpu -x -q \
    --timeout 200 --timeout-method thread ) > $O/C_sa_tests.log 2>&1 || exit $?
( cd .wip2 && timeout -k 10 300 python -u -m pytest tests/test_configs_gpu.py -m gpu -x -q -k "c2 or C2 or c1 or C1" \
    --timeout 250 --timeout-method thread ) > $O/C_cfg_tests.log 2>&1 || exit $?
