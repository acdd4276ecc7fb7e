#!/bin/bash
# round 3, GPU session 15: phase timers of k_sa_lds_fast (diagnostic build in .wip3)
set -o pipefail
O=$PWD/gpurun_out; mkdir -p $O
( cd .wip3 && timeout -k 10 300 python -u tools/sa_lds_prof.py ) > $O/H_sa_lds_prof.log 2>&1 || exit $?
