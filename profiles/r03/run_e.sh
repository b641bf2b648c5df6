# Round 3, run E: per-wave DPP dot reductions in tail_reduce / dir_sweep (no LDS staging of history values),
# fence-free hand-off in the column-sum kernels, sampled S-LBFGS timing with counted rows; full GPU suite;
# bench lines and kernel traces of cfg 2, the 7500-row shard and cfg 4.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03e
mkdir -p $O
cd $R
timeout -k 10 90 ./profiles/micro/launch_floor > $O/launch_floor.txt 2>&1 || echo "launch_floor failed"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|passed|failed" $O/gpu_tests.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/bench_cfg2.json 2> $O/bench_cfg2.err && \
timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 20 > $O/bench_cfg2_s20.json 2> $O/bench_cfg2_s20.err && \
timeout -k 10 120 python -u bench.py --no-cpu-baseline --samples 7500 > $O/bench_7500.json 2> $O/bench_7500.err && \
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err && \
LBF_DIR_FUSED=0 timeout -k 10 200 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline > $O/bench_cfg4_nodir.json 2> $O/bench_cfg4_nodir.err && \
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline --comm1 > $O/bench_cfg4_comm1.json 2> $O/bench_cfg4_comm1.err && \
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline --comm1 --samples 7500 --slbfgs-b 32 --slbfgs-bh 16 > $O/bench_cfg4_rank8.json 2> $O/bench_cfg4_rank8.err
echo "bench rc=$?"
cd /tmp && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --steps 3 --warmup 1 --no-cpu-baseline > $O/kt4.json 2> $O/kt4.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500.json 2> $O/kt7500.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt60000 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 50 > $O/kt60000.json 2> $O/kt60000.err && \
cd $R && python3 profiles/kstats_live.py $O/kt4/run_kernel_trace.csv --out $O/kt4_live.csv > /dev/null && \
python3 profiles/kstats_live.py --spec $O/kt7500/run_kernel_trace.csv --out $O/kt7500_live.csv > /dev/null && \
python3 profiles/kstats_live.py --spec $O/kt60000/run_kernel_trace.csv --out $O/kt60000_live.csv > /dev/null
echo "rc=$?"
