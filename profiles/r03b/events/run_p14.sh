# device-scope release on the library's events (profiling marks, twin fork / join): S-LBFGS + DP suites,
# then A/B against the system-scope default (LBF_EVENT_SYSTEM_RELEASE=1) on cfg 2 (driver shape, 400) and cfg 4
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03p14
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "slbfgs or dp or ranks or graph or combine or spec or fused" > $O/tests.log 2>&1 || { echo "tests failed"; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B() { n=$1; e=$2; shift 2; env $e timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; exit 1; }; }
B s20_dev LBF_X=0 --steps 20 --warmup 5 && B s20_sys LBF_EVENT_SYSTEM_RELEASE=1 --steps 20 --warmup 5 && \
B s20_dev2 LBF_X=0 --steps 20 --warmup 5 && B s20_sys2 LBF_EVENT_SYSTEM_RELEASE=1 --steps 20 --warmup 5 && \
B s400_dev LBF_X=0 && B s400_sys LBF_EVENT_SYSTEM_RELEASE=1 && \
B c4_dev LBF_X=0 --solver slbfgs --steps 8 --warmup 2 && B c4_sys LBF_EVENT_SYSTEM_RELEASE=1 --solver slbfgs --steps 8 --warmup 2
echo "rc=$?"
