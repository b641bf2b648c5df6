# Round 3, run N: the direct-operand 32x128 forward GEMM (gemm_direct_kernel): bitwise test against the LDS-DMA
# kernel, parity suites, 7500-row shard and cfg-4 benches direct vs LDS-DMA, kernel trace at 7500.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03n
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py -q -x -m gpu --timeout 120 --timeout-method thread -k "direct or slbfgs" > $O/direct_tests.log 2>&1 || { echo "direct tests failed"; tail -30 $O/direct_tests.log; exit 1; }
tail -1 $O/direct_tests.log
timeout -k 10 600 python -u -m pytest tests/ -q -x -m gpu --timeout 120 --timeout-method thread -k "parity or fullsize or spec or slbfgs or ranks" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp
for v in direct lds; do
  case $v in direct) E="LBF_GEMM_DIRECT=1";; lds) E="LBF_GEMM_DIRECT=0";; esac
  env $E timeout -k 10 120 python3 $R/bench.py --samples 7500 --no-cpu-baseline > $O/bench_7500_$v.json 2> $O/bench_7500_$v.err || exit 1
  env $E timeout -k 10 200 python3 $R/bench.py --solver slbfgs --steps 4 --warmup 2 --no-cpu-baseline > $O/cfg4_$v.json 2> $O/cfg4_$v.err || exit 1
done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500.json 2> $O/kt7500.err || exit 1
cd $R
python3 profiles/kstats_live.py --spec $O/kt7500/run_kernel_trace.csv --out $O/kt7500_live.csv
echo "rc=$?"
