# Two-loop microbench at cfg-5 n (fused tail on/off), per-rank shard sizes, cfg 3.
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 240 python -u bench_two_loop.py > $O/two_loop.jsonl 2> $O/two_loop.err && \
LBF_FUSED_TAIL=0 timeout -k 10 240 python -u bench_two_loop.py --m 10,20 > $O/two_loop_nofuse.jsonl 2> $O/two_loop_nofuse.err && \
for s in 7500 15000 30000; do timeout -k 10 120 python -u bench.py --samples $s --no-cpu-baseline > $O/bench_s$s.json 2> $O/bench_s$s.err || exit 1; done && \
timeout -k 10 120 python -u bench.py --dims 784,128,64,10 --acts relu,relu,linear --m 20 --no-cpu-baseline > $O/bench_cfg3.json 2> $O/bench_cfg3.err
echo "rc=$?"
