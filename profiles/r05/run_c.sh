#!/bin/bash
# round 5, run C: the 32 x 128 loop decomposition with the wave-split-K direct-load form
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05c
mkdir -p $O
cd $R
timeout -k 10 120 ./profiles/micro/loop32 > $O/loop32.txt 2>&1; echo "loop32 rc $?"; cat $O/loop32.txt
