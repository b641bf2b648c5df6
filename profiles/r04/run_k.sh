#!/bin/bash
# round 4, run K: the grouped dW1+dW0 launch (S-LBFGS minibatches): suite, then cfg 4 A/B against
# LBF_NO_GROUP=1 (two runs each, interleaved), and a kernel trace of the grouped route.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04k
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
B() { n=$1; shift; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; tail -1 $O/$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d.get('kernel_ms_per_step'))"; }
B cfg4_group_a --solver slbfgs --steps 6 --no-cpu-baseline
LBF_NO_GROUP=1 B cfg4_sep_a --solver slbfgs --steps 6 --no-cpu-baseline
B cfg4_group_b --solver slbfgs --steps 6 --no-cpu-baseline
LBF_NO_GROUP=1 B cfg4_sep_b --solver slbfgs --steps 6 --no-cpu-baseline
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --no-cpu-baseline --steps 3 --warmup 1 > $O/kt4.json 2> $O/kt4.err || { echo "prof failed"; exit 1; }
cd $R
python3 profiles/kstats_live.py $O/kt4/run_kernel_trace.csv --out $O/kt4_live.csv || { echo "kstats failed"; exit 1; }
echo "run k ok"
