R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 240 python -u bench_two_loop.py > $O/two_loop.jsonl 2> $O/two_loop.err
echo "rc=$?"
