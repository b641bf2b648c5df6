# Round 3, run A: launch-floor microbench, the new multi-rank tests (in-process rank group), the full GPU
# suite, then bench lines: cfg 2 (Wolfe, Armijo), the reference's deep GPU config (784-256-128-64-10,
# m = 10 / 100, Armijo + CUDA init = its main_gpu_deep.cpp), cfg 4 single and through a 1-rank communicator.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03a
mkdir -p $O
cd $R
timeout -k 10 60 ./profiles/micro/launch_floor > $O/launch_floor.txt 2>&1 || { echo "launch_floor failed"; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_ranks.py tests/test_gpu_dp.py -x -v --timeout 240 --timeout-method thread > $O/ranks_tests.log 2>&1
rc=$?; echo "ranks tests rc=$rc"; tail -3 $O/ranks_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -5 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/bench_cfg2.json 2> $O/bench_cfg2.err && \
timeout -k 10 120 python -u bench.py --no-cpu-baseline --line-search armijo --init cuda > $O/bench_cfg2_armijo.json 2> $O/bench_cfg2_armijo.err && \
timeout -k 10 120 python -u bench.py --no-cpu-baseline --dims 784,256,128,64,10 --acts relu,relu,relu,linear --m 10 --line-search armijo --init cuda > $O/bench_deep_m10_armijo.json 2> $O/bench_deep_m10_armijo.err && \
timeout -k 10 120 python -u bench.py --no-cpu-baseline --dims 784,256,128,64,10 --acts relu,relu,relu,linear --m 100 --steps 200 --line-search armijo --init cuda > $O/bench_deep_m100_armijo.json 2> $O/bench_deep_m100_armijo.err && \
timeout -k 10 120 python -u bench.py --no-cpu-baseline --dims 784,256,128,64,10 --acts relu,relu,relu,linear --m 10 > $O/bench_deep_m10_wolfe.json 2> $O/bench_deep_m10_wolfe.err && \
timeout -k 10 120 python -u bench.py --no-cpu-baseline --samples 7500 > $O/bench_7500.json 2> $O/bench_7500.err && \
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err && \
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline --comm1 > $O/bench_cfg4_comm1.json 2> $O/bench_cfg4_comm1.err
echo "bench rc=$?"
