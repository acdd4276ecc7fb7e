#!/bin/bash
# round 3, GPU session 11 (re-entry): full record at HEAD — parity tests, smoke, bench, kernel-trace summary
set -o pipefail
STEPS="tests smoke bench prof" bash tools/gpu_check.sh || exit $?
