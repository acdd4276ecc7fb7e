#!/bin/bash
# round 3, GPU session 1: parity tests, smoke, bench, then SA layout probe (cone vs rec)
set -o pipefail
O=gpurun_out; mkdir -p $O
STEPS="tests smoke bench" bash tools/gpu_check.sh || exit $?
SA_RS=1024,4096,16384 SA_LAYOUTS=cone,rec SA_K=1000 timeout -k 10 300 python -u tools/sa_scale.py > $O/sa_scale.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/sa_probe3.py > $O/sa_probe3.log 2>&1 || exit $?
