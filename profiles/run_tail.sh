# Tail rework check: fused-tail parity tests, per-rank and cfg-2 benches, phase stamps.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused_tail or speculative or wolfe_trajectory or slbfgs" tests/test_gpu_dp.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tail.log 2>&1 && \
timeout -k 10 120 python -u bench.py --samples 7500 --no-cpu-baseline --steps 100 > $O/bench_7500.json 2> $O/bench_7500.err && \
timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 100 > $O/bench.json 2> $O/bench.err && \
KT_N=7500 timeout -k 10 120 python -u profiles/ktrace.py > $O/ktrace_7500.txt 2>&1
echo "rc=$?"
