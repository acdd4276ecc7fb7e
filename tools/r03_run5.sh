#!/bin/bash
# round 3, GPU session 5: same-box A/B of the tree (A) against the .wip experiment copy (B):
# HPR update single-buffered at 2 workgroups per CU (B) vs double-buffered (A); SA speculative
# batches in half-full waves (B, kernel option spec_half) vs full waves
set -o pipefail
O=$PWD/gpurun_out; mkdir -p $O
ONLY_F32=1 timeout -k 10 120 python -u tools/hpr_time.py > $O/A_hpr_time.log 2>&1 || exit $?
( cd .wip && ONLY_F32=1 timeout -k 10 120 python -u tools/hpr_time.py ) > $O/B_hpr_time.log 2>&1 || exit $?
( cd .wip && timeout -k 10 300 python -u -m pytest tests/test_hpr_q_gpu.py tests/test_hpr_gpu.py -m gpu -x -q \
    --timeout 120 --timeout-method thread ) > $O/B_hpr_tests.log 2>&1 || exit $?
( cd .wip && timeout -k 10 400 python -u -m pytest tests/test_sa_gpu.py -m gpu -x -q -k "cone_layout" \
    --timeout 120 --timeout-method thread ) > $O/B_sa_tests.log 2>&1 || exit $?
( cd .wip && SA_RS=1024,4096,16384 SA_LAYOUTS=rec SA_KERNELS='{};{"spec_half": true}' SA_K=1000 \
    timeout -k 10 300 python -u tools/sa_scale.py ) > $O/B_sa_scale.log 2>&1 || exit $?
