#!/bin/bash
# round 4, run ZB: the final tree (after the row head partial-store split): whole suite, smoke, the driver-shape and
# 400-iteration cfg 2 lines, the 7500-row shard (single and 1-rank communicator), cfg 4
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04zb
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $O/smoke.log
B() { n=$1; shift; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'))"; }
B bench_driver --steps 20 --warmup 5
B bench_400 --steps 400 --no-cpu-baseline
B bench_7500 --steps 400 --samples 7500 --no-cpu-baseline
B bench_7500_comm1 --steps 400 --samples 7500 --no-cpu-baseline --comm1
B bench_cfg4 --solver slbfgs --steps 6
echo "run zb ok"
