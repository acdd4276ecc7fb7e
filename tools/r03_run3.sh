#!/bin/bash
# round 3, GPU session 3: parity tests, LDS-kernel probe, counter passes
set -o pipefail
O=gpurun_out; mkdir -p $O
STEPS="tests" bash tools/gpu_check.sh || exit $?
grep -q " passed" $O/pytest_gpu.log || exit 1
timeout -k 10 300 python -u tools/sa_probe3.py > $O/sa_probe3.log 2>&1 || exit $?
STEPS="sq pmc" bash tools/gpu_check.sh || exit $?
