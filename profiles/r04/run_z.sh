#!/bin/bash
# round 4, run Z: the row head's phase timestamps on config 4's minibatch (debug build)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04z
mkdir -p $O
cd $R
timeout -k 10 200 python -u profiles/ktrace_rowhead.py > $O/ktrace_rowhead.txt 2> $O/ktrace_rowhead.err || { echo "failed"; tail -5 $O/ktrace_rowhead.err; exit 1; }
cat $O/ktrace_rowhead.txt
echo "run z ok"
