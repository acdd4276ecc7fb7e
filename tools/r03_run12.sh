#!/bin/bash
# round 3, GPU session 12: the new init_generator test; SA_RRG.py's own problem (n=1e4, d=4, p=3, c=1)
# run towards consensus on 64 distinct graphs for up to 900 s (progress per chunk)
set -o pipefail
O=$PWD/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_hpr_q_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "init" > $O/E_hpr_init.log 2>&1 || exit $?
timeout -k 10 960 python -u tools/sa_cons_probe.py 10000 64 900 > $O/E_sa_cons_1e4.log 2>&1 || exit $?
