#!/bin/bash
# round 3, GPU session 22: SA_RRG.py's own problem (n=1e4, d=4, p=3, c=1) towards consensus on 64 distinct
# graphs with the paired LDS step, up to 1000 s (progress per chunk)
set -o pipefail
O=$PWD/gpurun_out; mkdir -p $O
timeout -k 10 1080 python -u tools/sa_cons_probe.py 10000 64 1000 > $O/O_sa_cons_1e4.log 2>&1 || exit $?
