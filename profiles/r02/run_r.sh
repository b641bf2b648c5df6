# Round 2, run R: EPI_DX epilogue with its act' operand loaded per (tm, tn) block before use: parity
# subset, cfg 3 A/B against build/ab (same cfg-3 route otherwise), cfg 4 and cfg 5 benches.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02r
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py tests/test_gpu_dp.py tests/test_gpu_fold.py -m gpu -q -x -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
AB=$R/lbfgs-ffnn_amd/build/ab/liblbfgs_amd.so
NEW=$R/lbfgs-ffnn_amd/build/liblbfgs_amd.so
for rep in 1 2; do
  for v in ab new; do
    L=$AB; [ $v = new ] && L=$NEW
    LBF_LIB_PATH=$L timeout -k 10 120 python -u bench.py --dims 784,128,64,10 --acts relu,relu,linear --m 20 --no-cpu-baseline > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit 1
  done
done
timeout -k 10 300 python -u bench.py --solver slbfgs --steps 6 --warmup 1 --no-cpu-baseline > $O/c4_new.json 2> $O/c4_new.err || exit 1
timeout -k 10 300 python -u bench.py --dims 4096,2048,1024,1 --acts relu,relu,linear --m 50 --samples 1000000 --data regression --steps 5 --warmup 2 --no-cpu-baseline > $O/c5_new.json 2> $O/c5_new.err || exit 1
echo "rc=0"
