# Round 2, run H: 8-wave (two k-group) LDS-DMA kernel for 32 x 128 tiles: full GPU suite, shard bench,
# cfg-2 bench, cfg-4 bench, kernel traces of the shard.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02h
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u bench.py --samples 7500 --no-cpu-baseline > $O/bench_7500.json 2> $O/bench_7500.err && \
timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/bench_cfg2.json 2> $O/bench_cfg2.err && \
timeout -k 10 300 python -u bench.py --solver slbfgs --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err && \
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500.json 2> $O/kt7500.err && \
cd $R && python3 profiles/kstats_live.py $O/kt7500/run_kernel_trace.csv --out $O/kt7500_live.csv > /dev/null
echo "rc=$?"
