# S-LBFGS epoch graphs: the new tests + the S-LBFGS suites, then cfg 4 graph / eager / anchor-precompute.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03p3
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_slbfgs_graph.py -x -v --timeout 120 --timeout-method thread > $O/graph_tests.log 2>&1 && \
LBF_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --solver slbfgs --steps 6 --warmup 2 --no-cpu-baseline > $O/cfg4_graph.json 2> $O/cfg4_graph.err && \
LBF_HOST_TIMING=1 LBF_SLBFGS_ANCHOR=1 timeout -k 10 200 python -u bench.py --solver slbfgs --steps 6 --warmup 2 --no-cpu-baseline > $O/cfg4_graph_pre.json 2> $O/cfg4_graph_pre.err && \
LBF_SLBFGS_GRAPH=0 timeout -k 10 200 python -u bench.py --solver slbfgs --steps 6 --warmup 2 --no-cpu-baseline > $O/cfg4_eager.json 2> $O/cfg4_eager.err && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "slbfgs or dp or ranks or fullsize or configs" > $O/slbfgs_tests.log 2>&1
echo "rc=$?"
