#!/bin/bash
# round 4, run R: the data-parallel tests after the SSE words moved into the reduce_all launch, then the
# 7500-row shard through the 1-rank communicator against the single route, interleaved
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04r
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_ranks.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_dp.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests_dp.log; exit 1; }
tail -1 $O/gpu_tests_dp.log
B() { n=$1; shift; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d.get('evals_per_iter'), d.get('kernel_ms_per_step'))"; }
B single_a --steps 400 --samples 7500 --no-cpu-baseline
B comm1_a --steps 400 --samples 7500 --no-cpu-baseline --comm1
B single_b --steps 400 --samples 7500 --no-cpu-baseline
B comm1_b --steps 400 --samples 7500 --no-cpu-baseline --comm1
echo "run r ok"
