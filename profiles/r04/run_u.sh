#!/bin/bash
# round 4, run U: speculation depth (iterations enqueued ahead of the line-search decision) in the driver's
# 20-iteration shape and over 400 iterations: a rejection drains every queued launch before the host-driven
# trial, so a shallower queue costs less per rejection but hides less host time
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04u
mkdir -p $O
cd $R
B() { n=$1; shift; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('evals_per_iter'))"; }
for rep in a b; do
  B drv_d3_$rep --steps 20 --warmup 5 --no-cpu-baseline
  LBF_SPEC_DEPTH=2 B drv_d2_$rep --steps 20 --warmup 5 --no-cpu-baseline
  LBF_SPEC_DEPTH=1 B drv_d1_$rep --steps 20 --warmup 5 --no-cpu-baseline
  LBF_SPEC_DEPTH=4 B drv_d4_$rep --steps 20 --warmup 5 --no-cpu-baseline
done
B s400_d3 --steps 400 --no-cpu-baseline
LBF_SPEC_DEPTH=2 B s400_d2 --steps 400 --no-cpu-baseline
LBF_SPEC_DEPTH=1 B s400_d1 --steps 400 --no-cpu-baseline
B s7500_d3 --steps 400 --samples 7500 --no-cpu-baseline
LBF_SPEC_DEPTH=2 B s7500_d2 --steps 400 --samples 7500 --no-cpu-baseline
echo "run u ok"
