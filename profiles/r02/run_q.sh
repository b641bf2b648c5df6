# Round 2, run Q: standalone head kernel with register-prefetched tiles and W (S-LBFGS minibatches): S-LBFGS /
# config / parity tests, cfg-4 bench A/B against build/ab, kernel trace of the new cfg-4 run.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02q
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_dp.py tests/test_gpu_fullsize.py tests/test_gpu_hvp.py -m gpu -q -x -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
AB=$R/lbfgs-ffnn_amd/build/ab/liblbfgs_amd.so
NEW=$R/lbfgs-ffnn_amd/build/liblbfgs_amd.so
for rep in 1 2; do
  for v in ab new; do
    L=$AB; [ $v = new ] && L=$NEW
    LBF_SHOW_PLAN=1 LBF_LIB_PATH=$L timeout -k 10 300 python -u bench.py --solver slbfgs --steps 6 --warmup 1 --no-cpu-baseline > $O/c4_${v}_$rep.json 2> $O/c4_${v}_$rep.err || exit 1
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --steps 3 --warmup 1 --no-cpu-baseline > $O/kt4.json 2> $O/kt4.err && \
cd $R && python3 profiles/kstats_live.py $O/kt4/run_kernel_trace.csv --out $O/kt4_live.csv > /dev/null
echo "rc=$?"
