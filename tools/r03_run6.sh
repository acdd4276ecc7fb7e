#!/bin/bash
# round 3, GPU session 6: q-layout HPR update A (tree: two buffers) / B (.wip: one buffer, 2 WGs per CU);
# phase timers of the speculative SA kernel (.wip2 diagnostic build, -DMJX_SA_PROF)
set -o pipefail
O=$PWD/gpurun_out; mkdir -p $O
timeout -k 10 120 python -u tools/hpr_q_time.py > $O/A_hpr_q_time.log 2>&1 || exit $?
( cd .wip && timeout -k 10 120 python -u tools/hpr_q_time.py ) > $O/B_hpr_q_time.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/hpr_q_time.py > $O/A2_hpr_q_time.log 2>&1 || exit $?
( cd .wip2 && SA_RS=1024,4096,16384 timeout -k 10 300 python -u tools/sa_prof.py ) > $O/C_sa_prof.log 2>&1 || exit $?
