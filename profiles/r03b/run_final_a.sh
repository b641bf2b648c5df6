# Round 3 (second session) evidence on the committed tree, part A: full GPU suite, smoke, the default bench
# line (with its CPU baseline), the driver's 20-step shape, Armijo, deep configs, cfg 3, m = 100, shards, cfg 4.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03fa
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/ -q -m gpu --timeout 120 --timeout-method thread > $O/final_gpu_tests.log 2>&1 || { echo "tests failed"; tail -20 $O/final_gpu_tests.log; exit 1; }
tail -1 $O/final_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/final_smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/final_smoke.log; exit 1; }
tail -1 $O/final_smoke.log
B() { n=$1; shift; timeout -k 10 200 python -u bench.py "$@" > $O/final_$n.json 2> $O/final_$n.err || { echo "bench $n failed"; tail -3 $O/final_$n.err; exit 1; }; }
B bench_cfg2_s20 --steps 20 --warmup 5
B bench_cfg2 --no-cpu-baseline
B bench_cfg2_armijo --line-search armijo --no-cpu-baseline
B bench_deep_m10 --dims 784,256,128,64,10 --acts relu,relu,relu,linear --m 10 --line-search armijo --no-cpu-baseline
B bench_deep_m100 --dims 784,256,128,64,10 --acts relu,relu,relu,linear --m 100 --line-search armijo --no-cpu-baseline
B bench_cfg3 --dims 784,128,64,10 --acts relu,relu,linear --m 20 --no-cpu-baseline
B bench_m100 --m 100 --no-cpu-baseline
B bench_7500 --samples 7500 --no-cpu-baseline
B bench_15000 --samples 15000 --no-cpu-baseline
B bench_30000 --samples 30000 --no-cpu-baseline
B bench_cfg4 --solver slbfgs --steps 8 --warmup 2
echo "rc=$?"
