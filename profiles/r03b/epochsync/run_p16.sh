# S-LBFGS epoch start without a host synchronisation (pinned index staging): suites, cfg 4 A/B
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03p16
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "slbfgs or dp or ranks or graph or combine or fullsize or configs" > $O/tests.log 2>&1 || { echo "tests failed"; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B() { n=$1; e=$2; shift 2; env $e timeout -k 10 200 python -u bench.py --no-cpu-baseline --solver slbfgs --steps 8 --warmup 2 "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; exit 1; }; }
B nosync1 LBF_X=0 && B sync1 LBF_SLBFGS_EPOCH_SYNC=1 && B nosync2 LBF_X=0 && B sync2 LBF_SLBFGS_EPOCH_SYNC=1
echo "rc=$?"
