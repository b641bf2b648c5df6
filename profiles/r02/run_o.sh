# Round 2, run O: forward tile by estimated launch time (Mlp::plan cost model): parity subset and the
# bench at the 1/2/4/8-rank shard sizes plus 40000 rows.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02o
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fold.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py tests/test_gpu_dp.py -m gpu -q -x -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
for S in 7500 15000 30000 40000 60000; do
  LBF_SHOW_PLAN=1 timeout -k 10 120 python -u bench.py --samples $S --no-cpu-baseline > $O/s${S}.json 2> $O/s${S}.err || exit 1
done
echo "rc=0"
