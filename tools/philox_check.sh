#!/bin/bash
# The Philox (non-parity) SA mode on the GPU: its parity tests, the SA GPU
# tests, and configs[1]'s throughput in both streams (tools/sa_scale.py).
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_sa_philox_gpu.py tests/test_sa_gpu.py tests/test_sa_multi_gpu.py tests/test_sa_script_size_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_sa.log 2>&1 || exit $?
SA_RS=4096 SA_K=2000 SA_LAYOUTS=rec,cone timeout -k 10 300 python -u tools/sa_scale.py > $OUT/c2_rng.log 2>&1 || exit $?
SA_RS=4096 SA_K=2000 SA_LAYOUTS=rec,cone SA_RNG=philox timeout -k 10 300 python -u tools/sa_scale.py >> $OUT/c2_rng.log 2>&1
