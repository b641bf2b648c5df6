# final tree (free-running twin on by default): full GPU suite, smoke, the default bench line, cfg 4
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03ff
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/ -q -m gpu --timeout 120 --timeout-method thread > $O/final_gpu_tests.log 2>&1 || { echo "tests failed"; tail -20 $O/final_gpu_tests.log; exit 1; }
tail -1 $O/final_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/final_smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/final_smoke.log; exit 1; }
tail -1 $O/final_smoke.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/final_bench_cfg2_s20.json 2> $O/final_bench_cfg2_s20.err && \
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 8 --warmup 2 > $O/final_bench_cfg4.json 2> $O/final_bench_cfg4.err
echo "rc=$?"
