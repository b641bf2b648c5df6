# Round 2, run L: 64 x 128 forward tiles for 8k-32k-row shards: forward-route parity, fold / full-size /
# DP tests, A/B against build/ab at the 1/2/4/8-rank shard sizes, kernel trace of the 15000-row shard.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02l
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fold.py tests/test_gpu_dp.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py -m gpu -q -x -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
AB=$R/lbfgs-ffnn_amd/build/ab/liblbfgs_amd.so
NEW=$R/lbfgs-ffnn_amd/build/liblbfgs_amd.so
for S in 15000 30000 7500 60000; do
  for v in ab new; do
    L=$AB; [ $v = new ] && L=$NEW
    LBF_LIB_PATH=$L timeout -k 10 120 python -u bench.py --samples $S --no-cpu-baseline > $O/s${S}_${v}.json 2> $O/s${S}_${v}.err || exit 1
  done
done
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt15000 -o run -- python3 $R/bench.py --samples 15000 --no-cpu-baseline --steps 50 > $O/kt15000.json 2> $O/kt15000.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt30000 -o run -- python3 $R/bench.py --samples 30000 --no-cpu-baseline --steps 50 > $O/kt30000.json 2> $O/kt30000.err && \
cd $R && python3 profiles/kstats_live.py $O/kt15000/run_kernel_trace.csv --out $O/kt15000_live.csv > /dev/null && \
python3 profiles/kstats_live.py $O/kt30000/run_kernel_trace.csv --out $O/kt30000_live.csv > /dev/null
echo "rc=$?"
