#!/bin/bash
# round 4, run ZA: the row head after its partial-row store split: phase marks, the S-LBFGS tests, cfg 4 x2
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04za
mkdir -p $O
cd $R
timeout -k 10 200 python -u profiles/ktrace_rowhead.py > $O/ktrace_rowhead.txt 2> $O/ktrace_rowhead.err || { echo "ktrace failed"; tail -5 $O/ktrace_rowhead.err; exit 1; }
cat $O/ktrace_rowhead.txt
timeout -k 10 500 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_slbfgs_run.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_dp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
B() { n=$1; shift; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('kernel_ms_per_step',{}).get('loss[0]'))"; }
B cfg4_a --solver slbfgs --steps 6 --no-cpu-baseline
B cfg4_b --solver slbfgs --steps 6 --no-cpu-baseline
echo "run za ok"
