#!/bin/bash
# round 3, GPU session 2: parity tests, then the counter passes (SQ; FETCH/WRITE incl. the ER sweeps)
set -o pipefail
O=gpurun_out; mkdir -p $O
STEPS="tests sq pmc" bash tools/gpu_check.sh || exit $?
