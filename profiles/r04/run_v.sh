#!/bin/bash
# round 4, run V: the suite after the line-search wait reductions (status read inside the drain, a Wolfe
# retry's backward enqueued with its loss-only forward), then the driver's shape A/B (LBF_SPEC_GRAD=0)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04v
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $O/smoke.log
B() { n=$1; shift; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('evals_per_iter'), d.get('loss_only_trials_per_iter'))"; }
for rep in a b c; do
  B drv_new_$rep --steps 20 --warmup 5 --no-cpu-baseline
  LBF_SPEC_GRAD=0 B drv_old_$rep --steps 20 --warmup 5 --no-cpu-baseline
done
B s400_new --steps 400 --no-cpu-baseline
LBF_SPEC_GRAD=0 B s400_old --steps 400 --no-cpu-baseline
B bench_driver --steps 20 --warmup 5
echo "run v ok"
