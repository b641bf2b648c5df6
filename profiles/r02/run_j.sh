# Round 2, run J: S-LBFGS hipGraph epochs: S-LBFGS tests, cfg-4 bench (graph / no graph), trace.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02j
mkdir -p $O
cd $R
true
rc=$?
echo "tests rc=$rc"
tail -3 $O/gpu_tests.log

timeout -k 10 300 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err && \
LBF_SLBFGS_GRAPH=0 timeout -k 10 300 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline > $O/bench_cfg4_nograph.json 2> $O/bench_cfg4_nograph.err
echo "rc=$?"
