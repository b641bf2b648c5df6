# Round-2 evidence (re-entry, after the S-LBFGS small-batch commits) on the committed tree: full GPU suite + smoke, PMC traffic of the headline kernel, the
# bench lines (cfg 2 with the CPU baseline, shards, cfg 3, m = 100, cfg 4, cfg 5), the two-loop
# microbench and rocprofv3 kernel traces of cfg 2 and the 7500-row shard.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02z
mkdir -p $O
cd $R
K="gemm_glds_kernel<2, 2, 2, 2, true, false, 3, false, 2"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -5 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
cd /tmp && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/pmc_fetch.json 2> $O/pmc_fetch.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/pmc_write.json 2> $O/pmc_write.err && \
python3 $R/profiles/collect_pmc.py $O/pmc_fetch $O/pmc_write --section "gemm_fwd[0]" --kernel "$K" --config 784,128,10:60000:1 --out $O/pmc_traffic.json && \
cp $O/pmc_traffic.json $R/profiles/pmc_traffic.json && cd $R && \
timeout -k 10 300 python -u bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err && \
timeout -k 10 120 python -u bench.py --samples 7500 --no-cpu-baseline > $O/bench_7500.json 2> $O/bench_7500.err && \
timeout -k 10 120 python -u bench.py --samples 15000 --no-cpu-baseline > $O/bench_15000.json 2> $O/bench_15000.err && \
timeout -k 10 120 python -u bench.py --samples 30000 --no-cpu-baseline > $O/bench_30000.json 2> $O/bench_30000.err && \
timeout -k 10 120 python -u bench.py --samples 7500 --no-cpu-baseline --comm1 > $O/bench_7500_comm1.json 2> $O/bench_7500_comm1.err && \
timeout -k 10 120 python -u bench.py --dims 784,128,64,10 --acts relu,relu,linear --m 20 --no-cpu-baseline > $O/bench_cfg3.json 2> $O/bench_cfg3.err && \
timeout -k 10 120 python -u bench.py --m 100 --steps 200 --no-cpu-baseline > $O/bench_m100.json 2> $O/bench_m100.err && \
timeout -k 10 300 python -u bench.py --solver slbfgs --steps 12 --warmup 1 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err && \
timeout -k 10 300 python -u bench.py --dims 4096,2048,1024,1 --acts relu,relu,linear --m 50 --samples 1000000 --data regression --steps 5 --warmup 2 --cpu-iters 2 --cpu-samples 400 > $O/bench_cfg5.json 2> $O/bench_cfg5.err && \
timeout -k 10 200 python -u bench_two_loop.py --m 10,20,50 > $O/two_loop.jsonl 2> $O/two_loop.err && \
cd /tmp && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt60000 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 50 > $O/kt60000.json 2> $O/kt60000.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500.json 2> $O/kt7500.err && \
python3 $R/profiles/kstats_live.py $O/kt60000/run_kernel_trace.csv --out $O/kt60000_live.csv > /dev/null && \
python3 $R/profiles/kstats_live.py $O/kt7500/run_kernel_trace.csv --out $O/kt7500_live.csv > /dev/null
echo "rc=$?"; [ -f $O/kt7500_live.csv ] || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --steps 3 --warmup 1 --no-cpu-baseline > $O/kt4.json 2> $O/kt4.err && \
cd $R && python3 profiles/kstats_live.py $O/kt4/run_kernel_trace.csv --out $O/kt4_live.csv > /dev/null
echo "rc4=$?"
