#!/bin/bash
# C2 (configs[1]) A/B: SA GPU tests on the product library, then tools/sa_scale.py
# at R=4096 (rec, cone) against each library of LIBS, twice, and the phase timers.
set -u
OUT=gpurun_out; mkdir -p $OUT
P=master-thesis-optimizing-initialization-in-graph-dynamics-from-ferromagnetism-to-opinion-consensus_amd/libmjx.so
timeout -k 10 600 python -u -m pytest tests/test_sa_gpu.py tests/test_sa_multi_gpu.py "tests/test_configs_gpu.py" -k "sa or c2 or spec or cone or rec" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
for rep in 1 2; do
  for lib in ${LIBS:-$P}; do
    SA_RS=4096 SA_K=2000 SA_LAYOUTS=rec,cone timeout -k 10 300 python -u tools/ab_lib.py $lib tools/sa_scale.py >> $OUT/c2_ab.log 2>&1 || exit $?
  done
done
if [ -f ab/libmjx_spprof.so ]; then
  SA_RS=4096 timeout -k 10 300 python -u tools/ab_lib.py ab/libmjx_spprof.so tools/sa_prof.py > $OUT/c2_prof.log 2>&1 || exit $?
fi
