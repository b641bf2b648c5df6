# Round 2, run E: S-LBFGS twin-stream evaluations (tests + cfg-4 bench with and without), dX tile.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02e
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -k "slbfgs or hvp or cfg4 or dp" > $O/gpu_tests.log 2>&1
echo "tests rc=$?"
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --solver slbfgs --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err && \
LBF_SLBFGS_TWIN=0 timeout -k 10 300 python -u bench.py --solver slbfgs --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_cfg4_notwin.json 2> $O/bench_cfg4_notwin.err && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_cfg4 -o run -- python3 $R/bench.py --no-cpu-baseline --solver slbfgs --steps 1 --warmup 1 > $O/kt_cfg4.json 2> $O/kt_cfg4.err && \
cd $R && python3 profiles/kstats_live.py $O/kt_cfg4/run_kernel_trace.csv --out $O/kt_cfg4_live.csv > /dev/null
echo "rc=$?"
