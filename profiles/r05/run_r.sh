#!/bin/bash
# round 5, run R: the cross-process RCCL tests with the 4-rank bench rehearsal.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05r
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest -v -s --timeout 600 --timeout-method thread tests/test_gpu_rccl_procs.py > $O/tests.log 2>&1; echo "tests rc $?"
grep -E "PASSED|FAILED|ERROR|bench --gpus" $O/tests.log | head -30
