# Round 2, run F: split-K plans (LBF_SHOW_PLAN) at cfg 2 / the 7500-row shard / cfg 3, the cfg-2 bench
# line with its CPU baseline, cfg-3 kernel trace, the two-loop microbench.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02f
mkdir -p $O
cd $R
LBF_SHOW_PLAN=1 timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 5 > $O/plan_cfg2.json 2> $O/plan_cfg2.err && \
LBF_SHOW_PLAN=1 timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 5 --samples 7500 > $O/plan_7500.json 2> $O/plan_7500.err && \
timeout -k 10 300 python -u bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err && \
timeout -k 10 200 python -u bench_two_loop.py --m 10,20,50 > $O/two_loop.jsonl 2> $O/two_loop.err && \
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_cfg3 -o run -- python3 $R/bench.py --no-cpu-baseline --dims 784,128,64,10 --acts relu,relu,linear --m 20 --steps 50 > $O/kt_cfg3.json 2> $O/kt_cfg3.err && \
cd $R && python3 profiles/kstats_live.py $O/kt_cfg3/run_kernel_trace.csv --out $O/kt_cfg3_live.csv > /dev/null
echo "rc=$?"
