#!/bin/bash
# Run AG (round 6): evidence on the final tree rebuilt in a re-created container, part 1 — the whole -m gpu suite, smoke, and the bench lines
# (cfg 2 driver shape with the CPU baseline, 400 iterations, the 7500-row shard single and through a 1-rank
# communicator, cfg 3, deep Armijo m = 10, cfg 4 with its CPU baseline, cfg 5).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ag
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|Error" $O/gpu_tests.log | head; tail -3 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $O/smoke.log
B() { n=$1; shift; timeout -k 10 240 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'), d.get('roofline',{}).get('avg_launch_us'), d.get('roofline',{}).get('traffic'), d.get('cpu_baseline',{}).get('value'))"; }
B bench_driver --steps 20 --warmup 5
B bench_400 --steps 400 --no-cpu-baseline
B bench_7500 --steps 400 --samples 7500 --no-cpu-baseline
B bench_7500_comm1 --steps 400 --samples 7500 --no-cpu-baseline --comm1
B bench_cfg3 --dims 784,128,64,10 --acts relu,relu,linear --m 20 --steps 200 --no-cpu-baseline
B bench_deep_m10 --dims 784,256,128,64,10 --acts relu,relu,relu,linear --line-search armijo --init cuda --steps 200 --no-cpu-baseline
B bench_cfg4 --solver slbfgs --steps 6
B bench_cfg5 --data regression --samples 1000000 --dims 4096,2048,1024,1 --acts relu,relu,linear --m 50 --steps 3 --warmup 1 --no-cpu-baseline --device-warmup 0
echo "run ag ok"
