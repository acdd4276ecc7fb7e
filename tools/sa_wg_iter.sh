#!/bin/bash
# One GPU call for a k_sa_lds_wg iteration: SA GPU tests, the probe, the phase
# timers (ab/libmjx_saprof.so) and two SQ counter passes (tools/sa_wg_pmc.sh).
set -u
PYTEST_PATHS="tests/test_sa_gpu.py tests/test_sa_script_size_gpu.py tests/test_sa_multi_gpu.py" STEPS="tests py" \
  TEST_TIMEOUT=600 PY="tools/sa_probe3.py --no-cone --pc 3,1 ;; tools/ab_lib.py ab/libmjx_saprof.so tools/sa_wg_prof.py" \
  bash tools/gpu_check.sh || exit $?
bash tools/sa_wg_pmc.sh
