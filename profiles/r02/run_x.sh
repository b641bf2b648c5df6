# Round 2, run X: re-entry check of the rebuilt tree: full GPU suite + smoke, cfg-2 bench, 7500-row shard
# (plain and --comm1), kernel trace of the shard.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02x
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/c2.json 2> $O/c2.err || exit 1
timeout -k 10 120 python -u bench.py --samples 7500 --no-cpu-baseline > $O/s7500.json 2> $O/s7500.err || exit 1
timeout -k 10 120 python -u bench.py --samples 7500 --no-cpu-baseline --comm1 > $O/s7500_comm1.json 2> $O/s7500_comm1.err || exit 1
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500.json 2> $O/kt7500.err && \
cd $R && python3 profiles/kstats_live.py $O/kt7500/run_kernel_trace.csv --out $O/kt7500_live.csv > /dev/null
echo "rc=$?"
