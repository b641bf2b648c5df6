# Full GPU test suite, per-rank / cfg-2 / cfg-5 benches.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u bench.py --samples 7500 --no-cpu-baseline --steps 100 > $O/bench_7500.json 2> $O/bench_7500.err && \
timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 100 > $O/bench.json 2> $O/bench.err && \
timeout -k 10 300 python -u bench.py --dims 4096,2048,1024,1 --acts relu,relu,linear --m 50 --samples 1000000 --data regression --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_cfg5.json 2> $O/bench_cfg5.err
echo "rc=$?"
