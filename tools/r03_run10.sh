#!/bin/bash
# round 3, GPU session 10: serialised phase timers of the speculative SA kernel (.wip2: every stamp drains
# the wave's memory counters, so each phase's exposed latency lands in its own bucket); LDS-resident SA
# kernel phase timers (.wip3)
set -o pipefail
O=$PWD/gpurun_out; mkdir -p $O
( cd .wip2 && SA_RS=4096,16384 timeout -k 10 300 python -u tools/sa_prof.py ) > $O/C_sa_prof5.log 2>&1 || exit $?
( cd .wip3 && timeout -k 10 300 python -u tools/sa_lds_prof.py ) > $O/D_sa_lds_prof.log 2>&1 || exit $?
