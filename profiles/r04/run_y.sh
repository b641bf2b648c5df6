#!/bin/bash
# round 4, run Y: the free-running twin posted 1 / 2 / 4 / 16 steps ahead (LBF_TWIN_AHEAD) on cfg 4, after
# the S-LBFGS tests under a deep look-ahead (same evaluations on the same inputs: bitwise the same results)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04y
mkdir -p $O
cd $R
LBF_TWIN_AHEAD=8 timeout -k 10 500 python -u -m pytest tests/test_gpu_slbfgs_run.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py -k "slbfgs or cfg4" -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_ahead8.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests_ahead8.log; exit 1; }
tail -1 $O/gpu_tests_ahead8.log
B() { n=$1; shift; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('final_loss'))"; }
for rep in a b; do
  B a1_$rep --solver slbfgs --steps 6 --no-cpu-baseline
  LBF_TWIN_AHEAD=2 B a2_$rep --solver slbfgs --steps 6 --no-cpu-baseline
  LBF_TWIN_AHEAD=4 B a4_$rep --solver slbfgs --steps 6 --no-cpu-baseline
  LBF_TWIN_AHEAD=16 B a16_$rep --solver slbfgs --steps 6 --no-cpu-baseline
done
echo "run y ok"
