#!/bin/bash
# round 4, run P: config 5 (4096-2048-1024-1, N = 1M, m = 50) and the 2- / 4-rank shards of config 2
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04p
mkdir -p $O
cd $R
B() { n=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'), d.get('roofline',{}).get('kernel'))"; }
B bench_cfg5 --dims 4096,2048,1024,1 --acts relu,relu,linear --m 50 --samples 1000000 --data regression --steps 5 --warmup 2 --cpu-iters 2 --cpu-samples 400 --device-warmup 3
B bench_15000 --steps 400 --samples 15000 --no-cpu-baseline
B bench_30000 --steps 400 --samples 30000 --no-cpu-baseline
B bench_7500 --steps 400 --samples 7500 --no-cpu-baseline
B bench_7500_comm1 --steps 400 --samples 7500 --no-cpu-baseline --comm1
echo "run p ok"
