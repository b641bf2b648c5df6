#!/bin/bash
# Round 6, run P: where the one-block history step's time goes at the two-loop shape (n = 10.49M):
# phase stamps (ktrace build) and per-kernel durations under rocprofv3 for m = 10 and m = 50.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
timeout -k 10 240 python -u profiles/r06/ktrace_hist.py --m 10,50 > $O/ktrace_hist.txt 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof50 -o run -- python3 bench_two_loop.py --m 50 --iters 10 > $O/two_loop50.jsonl 2> $O/two_loop50.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof10 -o run -- python3 bench_two_loop.py --m 10 --iters 10 > $O/two_loop10.jsonl 2> $O/two_loop10.err
