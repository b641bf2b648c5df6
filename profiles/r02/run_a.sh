# Round 2, run A: the full GPU suite (incl. the full-size oracle parity tests), the default bench line,
# and a rocprofv3 kernel trace of cfg 2 and the 7500-row shard.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02a
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "tests rc=$?"
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 120 python -u bench.py --samples 7500 --no-cpu-baseline > $O/bench_7500.json 2> $O/bench_7500.err && \
cd /tmp && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt60000 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 50 > $O/kt60000.json 2> $O/kt60000.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500.json 2> $O/kt7500.err && \
python3 $R/profiles/kstats_live.py $O/kt60000/run_kernel_trace.csv --out $O/kt60000_live.csv > /dev/null && \
python3 $R/profiles/kstats_live.py $O/kt7500/run_kernel_trace.csv --out $O/kt7500_live.csv > /dev/null
echo "rc=$?"
