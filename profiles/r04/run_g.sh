#!/bin/bash
# round 4, run G: split-K dX whose slabs the next dW GEMM sums in its B prologue (with act'); suite, cfg 4, cfg 2.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04g
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
B() { n=$1; shift; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; }
B bench_cfg4 --solver slbfgs --steps 6 --no-cpu-baseline
B bench_cfg4_b --solver slbfgs --steps 6 --no-cpu-baseline
B bench_driver --steps 20 --warmup 5
B bench_400 --steps 400 --no-cpu-baseline
B bench_7500 --steps 400 --samples 7500 --no-cpu-baseline
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --no-cpu-baseline --steps 3 --warmup 1 > $O/kt4.json 2> $O/kt4.err || { echo "prof failed"; exit 1; }
cd $R
python3 profiles/kstats_live.py $O/kt4/run_kernel_trace.csv --out $O/kt4_live.csv || { echo "kstats failed"; exit 1; }
echo "run g ok"
