# Round 2, run D: full GPU suite after the forward-only line-search trials, fused-head phase timeline
# (ktrace build), cfg 2 / cfg 3 bench lines.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02d
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "tests rc=$?"
tail -4 $O/gpu_tests.log
NS=60000,7500 timeout -k 10 120 python3 -u profiles/ktrace_gemm.py > $O/ktg.txt 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 120 python -u bench.py --dims 784,128,64,10 --acts relu,relu,linear --m 20 --no-cpu-baseline > $O/bench_cfg3.json 2> $O/bench_cfg3.err
echo "rc=$?"
