#!/bin/bash
# round 3, GPU session 31: member lanes by ds_permute instead of a mask scan (.wip5 = HEAD + that change):
# SA parity tests and step times there
set -o pipefail
O=$PWD/gpurun_out; mkdir -p $O
( cd .wip5 && timeout -k 10 600 python -u -m pytest tests/test_sa_gpu.py tests/test_sa_multi_gpu.py -m gpu -x -q \
    --timeout 200 --timeout-method thread ) > $O/W_sa_tests.log 2>&1 || exit $?
( cd .wip5 && timeout -k 10 300 python -u tools/sa_probe3.py ) > $O/W_sa_probe3.log 2>&1 || exit $?
