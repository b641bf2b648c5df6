# part B: rocprofv3 kernel traces + stats of the default bench line and the 7500-row shard, the PMC HBM-traffic
# passes behind the bench line's roofline.traffic, cfg 5, the two-loop microbench.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03fb
mkdir -p $O
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt60000 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 50 > $O/kt60000.json 2> $O/kt60000.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500.json 2> $O/kt7500.err || { echo "prof failed"; exit 1; }
cd $R
python3 profiles/kstats_live.py --spec $O/kt60000/run_kernel_trace.csv --out $O/kt60000_live.csv && \
python3 profiles/kstats_live.py --spec $O/kt7500/run_kernel_trace.csv --out $O/kt7500_live.csv || exit 1
K="gemm_glds_kernel<2, 2, 2, 2, true, false, 3, false, 2"
cd /tmp && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/pmc_fetch.json 2> $O/pmc_fetch.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/pmc_write.json 2> $O/pmc_write.err && \
python3 $R/profiles/collect_pmc.py $O/pmc_fetch $O/pmc_write --section "gemm_fwd[0]" --kernel "$K" --config 784,128,10:60000:1 --out $O/pmc_traffic.json || { echo "pmc failed"; exit 1; }
cd $R
timeout -k 10 300 python -u bench.py --dims 4096,2048,1024,1 --acts relu,relu,linear --m 50 --samples 1000000 --data regression --steps 5 --warmup 2 --cpu-iters 2 --cpu-samples 400 > $O/final_bench_cfg5.json 2> $O/final_bench_cfg5.err && \
timeout -k 10 200 python -u bench_two_loop.py --m 10,20,50 > $O/final_two_loop.jsonl 2> $O/final_two_loop.err
echo "rc=$?"
