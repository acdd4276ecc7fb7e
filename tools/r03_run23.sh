#!/bin/bash
# round 3, GPU session 23: record at HEAD after the LDS SA and HPR node-step work — every -m gpu test, smoke, bench, kernel trace
set -o pipefail
STEPS="tests smoke bench prof" bash tools/gpu_check.sh || exit $?
