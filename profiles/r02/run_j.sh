# Round 2, run J: S-LBFGS checks: tests, cfg-4 bench with and without the twin stream (12 epochs).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02j
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -k "slbfgs or hvp or cfg4 or dp or loss_grad" > $O/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -3 $O/gpu_tests.log

timeout -k 10 300 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err && \
LBF_SLBFGS_TWIN=0 timeout -k 10 300 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline > $O/bench_cfg4_notwin.json 2> $O/bench_cfg4_notwin.err
echo "rc=$?"
