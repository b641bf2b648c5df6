# ten-wave Gram sweep (2k live vectors spread evenly): full GPU suite, two-loop microbench A/B on one box
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03p9
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 200 python -u bench_two_loop.py --m 10,20,50 > $O/two_loop_w10.jsonl 2> $O/two_loop_w10.err && \
LBF_GRAM_W10=0 timeout -k 10 200 python -u bench_two_loop.py --m 10,50 > $O/two_loop_w8.jsonl 2> $O/two_loop_w8.err && \
timeout -k 10 200 python -u bench_two_loop.py --m 10,50 > $O/two_loop_w10b.jsonl 2> $O/two_loop_w10b.err
echo "rc=$?"
