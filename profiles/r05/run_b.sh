#!/bin/bash
# round 5, run B: the 32 x 128 k-tile loop decomposition (profiles/micro/loop32.hip) and the two-loop
# microbench under a kernel trace (durations without per-section events)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05b
mkdir -p $O
cd $R
timeout -k 10 120 ./profiles/micro/loop32 > $O/loop32.txt 2>&1; echo "loop32 rc $?"; cat $O/loop32.txt
timeout -k 10 300 python -u bench_two_loop.py --m 10,50 > $O/two_loop.jsonl 2> $O/two_loop.err; echo "two_loop rc $?"; cat $O/two_loop.jsonl | cut -c1-400
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt2l -o kt -- python3 $R/bench_two_loop.py --m 10,50 > $O/kt2l.log 2>&1; echo "kt rc $?"
find $O/kt2l -name "*kernel_stats.csv" | head -3
for f in $(find $O/kt2l -name "*kernel_stats.csv"); do head -12 $f | cut -c1-220; done
