# Round 2, run K: software-pipelined small-tile GEMM main loop (PIPE): parity subset, A/B against the
# committed build (build/ab) on the 7500-row shard, cfg 2 and cfg 4, shard kernel trace.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02k
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fold.py tests/test_gpu_dp.py tests/test_gpu_configs.py -m gpu -q -x -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
AB=$R/lbfgs-ffnn_amd/build/ab/liblbfgs_amd.so
NEW=$R/lbfgs-ffnn_amd/build/liblbfgs_amd.so
for rep in 1 2; do
  for v in ab new; do
    L=$AB; [ $v = new ] && L=$NEW
    LBF_LIB_PATH=$L timeout -k 10 120 python -u bench.py --samples 7500 --no-cpu-baseline --steps 300 > $O/s_${v}_$rep.json 2> $O/s_${v}_$rep.err || exit 1
  done
done
for v in ab new; do
  L=$AB; [ $v = new ] && L=$NEW
  LBF_LIB_PATH=$L timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/b_${v}.json 2> $O/b_${v}.err || exit 1
  LBF_LIB_PATH=$L timeout -k 10 300 python -u bench.py --solver slbfgs --steps 4 --warmup 1 --no-cpu-baseline > $O/c4_${v}.json 2> $O/c4_${v}.err || exit 1
done
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500.json 2> $O/kt7500.err && \
cd $R && python3 profiles/kstats_live.py $O/kt7500/run_kernel_trace.csv --out $O/kt7500_live.csv > /dev/null
echo "rc=$?"
