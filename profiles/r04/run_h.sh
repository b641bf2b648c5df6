#!/bin/bash
# round 4, run H: split-K dX into the dW B prologue: step-exact S-LBFGS parity, the chaotic one-epoch check
# (printed), the rest of the suite after it, cfg 4 / cfg 2 benches.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04h
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -k "slbfgs" -x -q --timeout 200 --timeout-method thread > $O/slbfgs_parity.log 2>&1 || { echo "slbfgs parity failed"; tail -30 $O/slbfgs_parity.log; exit 1; }
tail -1 $O/slbfgs_parity.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -k "cfg4" -q -s --timeout 250 --timeout-method thread > $O/cfg4_epoch.log 2>&1; echo "cfg4 epoch check rc=$?"; grep "cfg4 epoch loss" $O/cfg4_epoch.log
B() { n=$1; shift; timeout -k 10 200 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -3 $O/$n.err; exit 1; }; }
B bench_cfg4 --solver slbfgs --steps 6 --no-cpu-baseline
B bench_cfg4_b --solver slbfgs --steps 6 --no-cpu-baseline
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_fullsize.py::test_cfg4_slbfgs_one_epoch_full_size > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --no-cpu-baseline --steps 3 --warmup 1 > $O/kt4.json 2> $O/kt4.err || { echo "prof failed"; exit 1; }
cd $R
python3 profiles/kstats_live.py $O/kt4/run_kernel_trace.csv --out $O/kt4_live.csv || { echo "kstats failed"; exit 1; }
echo "run h ok"
