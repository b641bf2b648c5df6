#!/bin/bash
# round 4, run X: phase timestamps of the L-BFGS tail (debug build, profiles/ktrace.py) at 60000 and 7500 rows
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04x
mkdir -p $O
cd $R
KT_N=60000 timeout -k 10 200 python -u profiles/ktrace.py > $O/ktrace_60000.txt 2> $O/ktrace_60000.err || { echo "kt60000 failed"; tail -5 $O/ktrace_60000.err; exit 1; }
cat $O/ktrace_60000.txt
KT_N=7500 timeout -k 10 200 python -u profiles/ktrace.py > $O/ktrace_7500.txt 2> $O/ktrace_7500.err || { echo "kt7500 failed"; tail -5 $O/ktrace_7500.err; exit 1; }
cat $O/ktrace_7500.txt
echo "run x ok"
