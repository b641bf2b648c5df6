# eight-wave dir_sweep blocks (LBF_DIR_WAVES=8): S-LBFGS parity with it, cfg 4 A/B
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03p12
mkdir -p $O
cd $R
LBF_DIR_WAVES=8 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "slbfgs or graph or combine or fullsize" > $O/tests_w8.log 2>&1 || { echo "tests failed"; tail -20 $O/tests_w8.log; exit 1; }
tail -1 $O/tests_w8.log
B() { n=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --solver slbfgs --steps 8 --warmup 2 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { echo "$n failed"; exit 1; }; }
B w8 LBF_DIR_WAVES=8 && B w4 LBF_DIR_WAVES=4 && B w8b LBF_DIR_WAVES=8 && B w4b LBF_DIR_WAVES=4
echo "rc=$?"
