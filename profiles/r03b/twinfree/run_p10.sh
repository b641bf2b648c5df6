# free-running twin (per-step anchor buffers, no ev_free_ on the context stream): S-LBFGS suites, cfg 4 A/B
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03p10
mkdir -p $O
cd $R
LBF_SLBFGS_TWIN_FREE=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "slbfgs or dp or ranks or fullsize or configs or graph or combine" > $O/slbfgs_tests.log 2>&1 && \
LBF_SLBFGS_TWIN_FREE=1 LBF_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --solver slbfgs --steps 8 --warmup 2 --no-cpu-baseline > $O/cfg4_free.json 2> $O/cfg4_free.err && \
LBF_HOST_TIMING=1 LBF_SLBFGS_TWIN_FREE=0 timeout -k 10 200 python -u bench.py --solver slbfgs --steps 8 --warmup 2 --no-cpu-baseline > $O/cfg4_nofree.json 2> $O/cfg4_nofree.err && \
LBF_SLBFGS_TWIN_FREE=1 LBF_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --solver slbfgs --steps 8 --warmup 2 --no-cpu-baseline > $O/cfg4_free2.json 2> $O/cfg4_free2.err
echo "rc=$?"
