R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03q
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "slbfgs or dp or ranks or graph or combine" > $O/tests.log 2>&1 || { echo "tests failed"; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
LBF_SLBFGS_TWIN_FREE_MB=0 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "slbfgs_graph or test_slbfgs" > $O/tests_budget0.log 2>&1 || { echo "tests (budget 0) failed"; tail -20 $O/tests_budget0.log; exit 1; }
tail -1 $O/tests_budget0.log
timeout -k 10 200 python -u bench.py --no-cpu-baseline --solver slbfgs --steps 8 --warmup 2 > $O/cfg4.json 2> $O/cfg4.err
echo "rc=$?"
