#!/bin/bash
# round 3, GPU session 14: k_sa_lds_fast v2 (ballot sums, dedup at the last level only, prefetched rows)
set -o pipefail
O=$PWD/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sa_gpu.py tests/test_sa_multi_gpu.py -m gpu -x -q --timeout 200 \
    --timeout-method thread > $O/G_sa_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/sa_probe3.py > $O/G_sa_probe3.log 2>&1 || exit $?
