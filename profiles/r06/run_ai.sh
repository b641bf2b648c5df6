#!/bin/bash
# Run AI (round 6): evidence on the final tree after the early Armijo test (run AH ran the whole -m gpu suite on this
# code: 319 passed) — smoke, every bench line (cfg 2 driver shape with the CPU baseline, 400 iterations, the 7500-row
# shard single and through a 1-rank communicator, cfg 3, deep Armijo m = 10, cfg 4 with its CPU baseline, cfg 5),
# kernel traces of cfg 2 (driver shape) and the 7500-row shard with live statistics.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ai
mkdir -p $O
cd $R
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $O/smoke.log
B() { n=$1; shift; timeout -k 10 240 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('evals_per_iter'), d.get('roofline',{}).get('frac'), d.get('roofline',{}).get('avg_launch_us'), d.get('roofline',{}).get('traffic'), d.get('cpu_baseline',{}).get('value'))"; }
B bench_driver --steps 20 --warmup 5
B bench_400 --steps 400 --no-cpu-baseline
B bench_7500 --steps 400 --samples 7500 --no-cpu-baseline
B bench_7500_comm1 --steps 400 --samples 7500 --no-cpu-baseline --comm1
B bench_cfg3 --dims 784,128,64,10 --acts relu,relu,linear --m 20 --steps 200 --no-cpu-baseline
B bench_deep_m10 --dims 784,256,128,64,10 --acts relu,relu,relu,linear --line-search armijo --init cuda --steps 200 --no-cpu-baseline
B bench_cfg4 --solver slbfgs --steps 6
B bench_cfg5 --data regression --samples 1000000 --dims 4096,2048,1024,1 --acts relu,relu,linear --m 50 --steps 3 --warmup 1 --no-cpu-baseline --device-warmup 0
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt60000 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/kt60000.json 2> $O/kt60000.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500.json 2> $O/kt7500.err || { echo "prof failed"; exit 1; }
cd $R
python3 profiles/kstats_live.py --spec $O/kt60000/run_kernel_trace.csv --out $O/kt60000_live.csv && \
python3 profiles/kstats_live.py --spec $O/kt7500/run_kernel_trace.csv --out $O/kt7500_live.csv || echo "kstats failed"
head -4 $O/kt60000_live.csv
echo "run ai ok"
