#!/bin/bash
# A/B of the C5 binned sweep: ab/libmjx_head.so (previous commit) vs the tree's
# libmjx.so under phase-1/phase-2 knobs, alternating, on the same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  MJX_LIB=$PWD/ab/libmjx_head.so timeout -k 10 60 python3 tools/bin_exp.py 1e9 6 0 2>&1 | grep EXP | sed 's/^/head /' || exit 1
  for cfg in ${CFGS:-"4 4"}; do :; done
  for uc1 in ${UC1S:-4}; do for uc2 in ${UC2S:-4}; do
    MJX_BIN_UC1=$uc1 MJX_BIN_UC2=$uc2 timeout -k 10 60 python3 tools/bin_exp.py 1e9 6 0 2>&1 | grep EXP | sed "s/^/new uc1=$uc1 uc2=$uc2 /" || exit 1
  done; done
done
