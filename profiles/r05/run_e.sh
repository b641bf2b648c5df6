#!/bin/bash
# round 5, run E: the cfg-4 parity tests (first pair at the device's own FD points, ReLU epoch at 5 %, tanh epoch)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05e
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_gpu_fullsize.py -k "cfg4" > $O/cfg4.log 2>&1; echo "cfg4 rc $?"
grep -E "first pair|cfg4 |PASSED|FAILED|Error" $O/cfg4.log | head -30
