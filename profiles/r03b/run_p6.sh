# twin-stream enqueue on a helper host thread: S-LBFGS suites, then cfg 4 with / without it (same box)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03p6
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "slbfgs or dp or ranks or fullsize or configs or graph" > $O/slbfgs_tests.log 2>&1 && \
LBF_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --solver slbfgs --steps 6 --warmup 2 --no-cpu-baseline > $O/cfg4_thread.json 2> $O/cfg4_thread.err && \
LBF_HOST_TIMING=1 LBF_SLBFGS_TWIN_THREAD=0 timeout -k 10 200 python -u bench.py --solver slbfgs --steps 6 --warmup 2 --no-cpu-baseline > $O/cfg4_nothread.json 2> $O/cfg4_nothread.err && \
LBF_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --solver slbfgs --steps 6 --warmup 2 --no-cpu-baseline > $O/cfg4_thread2.json 2> $O/cfg4_thread2.err
echo "rc=$?"
