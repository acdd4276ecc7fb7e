#!/bin/bash
# round 3, GPU session 8: q-layout HPR update with double-buffered old rows (tree) -- parity + timing;
# finer phase timers of the speculative SA kernel (.wip2 diagnostic build)
set -o pipefail
O=$PWD/gpurun_out; mkdir -p $O
PYTEST_PATHS="tests/test_hpr_q_gpu.py tests/test_hpr_gpu.py tests/test_drop_in.py" STEPS="tests" bash tools/gpu_check.sh || exit $?
timeout -k 10 120 python -u tools/hpr_q_time.py > $O/A_hpr_q_time.log 2>&1 || exit $?
( cd .wip2 && SA_RS=1024,4096,16384 timeout -k 10 300 python -u tools/sa_prof.py ) > $O/C_sa_prof3.log 2>&1 || exit $?
