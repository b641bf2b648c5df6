# Full GPU test suite + per-rank and cfg-2 benches.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u bench.py --samples 7500 --no-cpu-baseline --steps 100 > $O/bench_7500.json 2> $O/bench_7500.err && \
timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 100 > $O/bench.json 2> $O/bench.err
echo "rc=$?"
