# Round-1 evidence: the default bench line (cfg 2, with the CPU baseline), the per-rank shard bench,
# rocprofv3 kernel traces of both (live-launch stats), the cfg-5 bench and the two-loop microbench.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R
timeout -k 10 300 python -u bench.py > $O/final_bench.json 2> $O/final_bench.err && \
timeout -k 10 120 python -u bench.py --samples 7500 --no-cpu-baseline > $O/final_bench_7500.json 2> $O/final_bench_7500.err && \
timeout -k 10 120 python -u bench.py --samples 15000 --no-cpu-baseline > $O/final_bench_15000.json 2> $O/final_bench_15000.err && \
timeout -k 10 120 python -u bench.py --samples 30000 --no-cpu-baseline > $O/final_bench_30000.json 2> $O/final_bench_30000.err && \
timeout -k 10 120 python -u bench.py --dims 784,128,64,10 --acts relu,relu,linear --m 20 --no-cpu-baseline > $O/final_bench_cfg3.json 2> $O/final_bench_cfg3.err && \
timeout -k 10 300 python -u bench.py --dims 4096,2048,1024,1 --acts relu,relu,linear --m 50 --samples 1000000 --data regression --steps 5 --warmup 2 --cpu-iters 2 --cpu-samples 400 > $O/final_bench_cfg5.json 2> $O/final_bench_cfg5.err && \
timeout -k 10 200 python -u bench_two_loop.py --m 10,20,50 > $O/final_two_loop.jsonl 2> $O/final_two_loop.err && \
cd /tmp && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fkt60000 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 50 > $O/fkt60000.json 2> $O/fkt60000.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fkt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/fkt7500.json 2> $O/fkt7500.err && \
python3 $R/profiles/kstats_live.py $O/fkt60000/run_kernel_trace.csv --out $O/fkt60000_live.csv > /dev/null && \
python3 $R/profiles/kstats_live.py $O/fkt7500/run_kernel_trace.csv --out $O/fkt7500_live.csv > /dev/null
echo "rc=$?"
