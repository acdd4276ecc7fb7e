#!/bin/bash
set -o pipefail
O=gpurun_out/r03; mkdir -p $O
timeout -k 10 300 python -u tools/sa_probe3.py 2>&1 | tee $O/sa_probe3.log || exit 1
timeout -k 10 200 python -u tools/sa_cons_probe.py 1000 2 2>&1 | tee $O/sa_cons_probe.log || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_sa_multi_gpu.py tests/test_sa_gpu.py 2>&1 | tee $O/sa_tests.log || exit 1
