# Round 3 (second session), first call: smoke, the default bench line, and a cfg-4 kernel trace whose
# per-stream gaps locate the inner step's idle time.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03p1
mkdir -p $O
cd $R
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/bench_s20.json 2> $O/bench_s20.err && \
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 4 --warmup 2 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err && \
cd /tmp && \
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --steps 2 --warmup 1 --no-cpu-baseline > $O/kt4.json 2> $O/kt4.err || { echo "failed"; exit 1; }
cd $R
python3 profiles/gaps.py --top 30 $O/kt4/run_kernel_trace.csv > $O/gaps_cfg4.txt
echo "rc=$?"
