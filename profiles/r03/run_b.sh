# Round 3, run B: the two-launch S-LBFGS history update (dir.hip): S-LBFGS parity tests, cfg-4 bench
# A/B against the three-launch route (LBF_DIR_FUSED=0), kernel traces of cfg 4 and of the 7500-row
# shard, and the step-0.01 NaN diagnostic (device vs oracle pair traces).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03b
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "slbfgs or cfg4 or fd_hvp or ranks or dp" > $O/slbfgs_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/slbfgs_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err && \
LBF_DIR_FUSED=0 timeout -k 10 200 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline > $O/bench_cfg4_nodir.json 2> $O/bench_cfg4_nodir.err && \
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline --comm1 > $O/bench_cfg4_comm1.json 2> $O/bench_cfg4_comm1.err && \
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline --comm1 --samples 7500 --slbfgs-b 32 --slbfgs-bh 16 > $O/bench_cfg4_rank8.json 2> $O/bench_cfg4_rank8.err && \
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline --comm1 --samples 15000 --slbfgs-b 64 --slbfgs-bh 32 > $O/bench_cfg4_rank4.json 2> $O/bench_cfg4_rank4.err && \
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline --comm1 --samples 30000 --slbfgs-b 128 --slbfgs-bh 64 > $O/bench_cfg4_rank2.json 2> $O/bench_cfg4_rank2.err && \
cd /tmp && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --steps 3 --warmup 1 --no-cpu-baseline > $O/kt4.json 2> $O/kt4.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500.json 2> $O/kt7500.err && \
cd $R && python3 profiles/kstats_live.py $O/kt4/run_kernel_trace.csv --out $O/kt4_live.csv > /dev/null && \
python3 profiles/kstats_live.py --spec $O/kt7500/run_kernel_trace.csv --out $O/kt7500_live.csv > /dev/null && \
timeout -k 10 300 python -u profiles/r03/diag_nan.py > $O/diag_nan.log 2>&1
echo "rc=$?"
