# gram_fin (unfused history path: column sums + last-block step) and the vectorised Gram sweep: GPU suite,
# the two-loop microbench, and cfg 4 with host-side enqueue timing.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03p2
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 200 python -u bench_two_loop.py --m 10,20,50 > $O/two_loop.jsonl 2> $O/two_loop.err && \
LBF_GRAM_FIN=0 LBF_GRAM_VEC=0 timeout -k 10 200 python -u bench_two_loop.py --m 10,50 > $O/two_loop_old.jsonl 2> $O/two_loop_old.err && \
LBF_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --solver slbfgs --steps 4 --warmup 2 --no-cpu-baseline > $O/cfg4_ht.json 2> $O/cfg4_ht.err
echo "rc=$?"
