# Two-loop history tests + the cfg-5-n two-loop microbenchmark.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "two_loop or wolfe or fused or speculative or slbfgs" -x -q --timeout 120 --timeout-method thread > $O/gpu_2loop.log 2>&1 && \
timeout -k 10 200 python -u bench_two_loop.py --m 10,20,50 > $O/two_loop.jsonl 2> $O/two_loop.err
echo "rc=$?"
