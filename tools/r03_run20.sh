#!/bin/bash
# round 3, GPU session 20: paired LDS SA phase timers, with and without the returning atomics at the last level (.wip4: timing only, results wrong)
set -o pipefail
O=$PWD/gpurun_out; mkdir -p $O
( cd .wip3 && timeout -k 10 300 python -u tools/sa_lds_prof.py ) > $O/M_prof_ret.log 2>&1 || exit $?
( cd .wip4 && timeout -k 10 300 python -u tools/sa_lds_prof.py ) > $O/M_prof_noret.log 2>&1 || exit $?
