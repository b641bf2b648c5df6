# Round 3, run C (= runs A + B, which found no box): launch-floor microbench; the multi-rank tests (in-process
# rank group) and the full GPU suite; bench lines: cfg 2 (Wolfe, Armijo + CUDA init), the reference's deep GPU
# config (784-256-128-64-10, m = 10 / 100), the 7500-row shard, cfg 4 (two-launch S-LBFGS update, A/B
# against the three-launch route, the 1-rank DP route, the per-rank slices of 2 / 4 / 8-rank runs); kernel
# traces of cfg 4 and the 7500-row shard; the step-0.01 NaN diagnostic.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03c
mkdir -p $O
cd $R
timeout -k 10 60 ./profiles/micro/launch_floor > $O/launch_floor.txt 2>&1 || { echo "launch_floor failed"; exit 1; }
timeout -k 10 200 python -u profiles/r03/dbg_armijo_ranks.py > $O/dbg_armijo.log 2>&1 || { echo "dbg failed"; tail -5 $O/dbg_armijo.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_ranks.py tests/test_gpu_dp.py -v --timeout 240 --timeout-method thread > $O/ranks_tests.log 2>&1
rc=$?; echo "ranks tests rc=$rc"; tail -3 $O/ranks_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread --ignore=tests/test_gpu_ranks.py > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -5 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/bench_cfg2.json 2> $O/bench_cfg2.err && \
timeout -k 10 120 python -u bench.py --no-cpu-baseline --line-search armijo --init cuda > $O/bench_cfg2_armijo.json 2> $O/bench_cfg2_armijo.err && \
timeout -k 10 120 python -u bench.py --no-cpu-baseline --dims 784,256,128,64,10 --acts relu,relu,relu,linear --m 10 --line-search armijo --init cuda > $O/bench_deep_m10_armijo.json 2> $O/bench_deep_m10_armijo.err && \
timeout -k 10 120 python -u bench.py --no-cpu-baseline --dims 784,256,128,64,10 --acts relu,relu,relu,linear --m 100 --steps 200 --line-search armijo --init cuda > $O/bench_deep_m100_armijo.json 2> $O/bench_deep_m100_armijo.err && \
timeout -k 10 120 python -u bench.py --no-cpu-baseline --dims 784,256,128,64,10 --acts relu,relu,relu,linear --m 10 > $O/bench_deep_m10_wolfe.json 2> $O/bench_deep_m10_wolfe.err && \
timeout -k 10 120 python -u bench.py --no-cpu-baseline --samples 7500 > $O/bench_7500.json 2> $O/bench_7500.err && \
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err && \
LBF_DIR_FUSED=0 timeout -k 10 200 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline > $O/bench_cfg4_nodir.json 2> $O/bench_cfg4_nodir.err && \
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline --comm1 > $O/bench_cfg4_comm1.json 2> $O/bench_cfg4_comm1.err && \
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline --comm1 --samples 7500 --slbfgs-b 32 --slbfgs-bh 16 > $O/bench_cfg4_rank8.json 2> $O/bench_cfg4_rank8.err && \
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline --comm1 --samples 15000 --slbfgs-b 64 --slbfgs-bh 32 > $O/bench_cfg4_rank4.json 2> $O/bench_cfg4_rank4.err && \
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline --comm1 --samples 30000 --slbfgs-b 128 --slbfgs-bh 64 > $O/bench_cfg4_rank2.json 2> $O/bench_cfg4_rank2.err
echo "bench rc=$?"
cd /tmp && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --steps 3 --warmup 1 --no-cpu-baseline > $O/kt4.json 2> $O/kt4.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500.json 2> $O/kt7500.err && \
cd $R && python3 profiles/kstats_live.py $O/kt4/run_kernel_trace.csv --out $O/kt4_live.csv > /dev/null && \
python3 profiles/kstats_live.py --spec $O/kt7500/run_kernel_trace.csv --out $O/kt7500_live.csv > /dev/null && \
timeout -k 10 400 python -u profiles/r03/diag_nan.py > $O/diag_nan.log 2>&1
echo "rc=$?"
