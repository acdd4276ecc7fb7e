#!/bin/bash
# SA GPU tests, the LDS probes at p=3 and p=c=1, the p=c=1 phase timers and configs[1]'s rate.
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_sa_philox_gpu.py tests/test_sa_gpu.py tests/test_sa_multi_gpu.py tests/test_sa_script_size_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_sa.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/sa_probe3.py --no-cone --pc "1,1;3,1" > $OUT/probe.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_lib.py ab/libmjx_saprof.so tools/sa_wg1_prof.py >> $OUT/probe.log 2>&1 && timeout -k 10 300 python -u tools/ab_lib.py ab/libmjx_saprof.so tools/sa_wg_prof.py >> $OUT/probe.log 2>&1 || exit $?
SA_RS=4096 SA_K=2000 SA_LAYOUTS=rec timeout -k 10 300 python -u tools/sa_scale.py >> $OUT/probe.log 2>&1
