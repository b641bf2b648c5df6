# Round 2, run G: m = 100 history step (LDS layout for k > 64): two-loop parity + trajectories, bench.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02g
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "tests rc=$?"
tail -3 $O/gpu_tests.log
timeout -k 10 200 python -u bench.py --m 100 --warmup 110 --no-cpu-baseline > $O/bench_m100.json 2> $O/bench_m100.err && \
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_m100 -o run -- python3 $R/bench.py --no-cpu-baseline --m 100 --warmup 110 --steps 100 > $O/kt_m100.json 2> $O/kt_m100.err && \
cd $R && python3 profiles/kstats_live.py $O/kt_m100/run_kernel_trace.csv --out $O/kt_m100_live.csv > /dev/null
echo "rc=$?"
