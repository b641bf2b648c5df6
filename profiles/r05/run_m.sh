#!/bin/bash
# round 5, run M: the rank-group tests rewritten around the non-chaotic window (first-pair snapshot) and the
# tanh epoch at a fixed 2 %, on the new head epilogue; the full-size S-LBFGS tests beside them.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05m
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_ranks.py tests/test_gpu_fullsize.py -k "slbfgs or cfg4" > $O/tests.log 2>&1; echo "tests rc $?"
grep -E "PASSED|FAILED|ERROR|cfg4|first pair" $O/tests.log | grep -v "^tests.*PASSED$" | head -40; grep -E "passed|failed" $O/tests.log | tail -2
