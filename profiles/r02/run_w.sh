# Round 2, run W: standalone head split over the hidden width for few-tile batches: full GPU suite,
# cfg-4 bench x2, the data-parallel route at the 8-rank shard (--comm1), cfg 2 control, cfg-4 kernel trace.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02w
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --solver slbfgs --steps 6 --warmup 1 --no-cpu-baseline > $O/c4_$rep.json 2> $O/c4_$rep.err || exit 1
done
timeout -k 10 120 python -u bench.py --samples 7500 --no-cpu-baseline --comm1 > $O/s7500_comm1.json 2> $O/s7500_comm1.err || exit 1
timeout -k 10 120 python -u bench.py --samples 15000 --no-cpu-baseline --comm1 > $O/s15000_comm1.json 2> $O/s15000_comm1.err || exit 1
timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/c2.json 2> $O/c2.err || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --steps 3 --warmup 1 --no-cpu-baseline > $O/kt4.json 2> $O/kt4.err && \
cd $R && python3 profiles/kstats_live.py $O/kt4/run_kernel_trace.csv --out $O/kt4_live.csv > /dev/null
echo "rc=$?"
