# Round 2, run AG: fused-tail slab reduction with 24 loads per column in flight when a segment has more than
# 32 split-K slabs (cfg 2: 82 slabs, one round instead of three): full GPU suite, cfg 2 A/B x3 (build/ab =
# previous commit), kernel trace of cfg 2.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02ag
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
AB="LBF_LIB_PATH=$R/lbfgs-ffnn_amd/build/ab/liblbfgs_amd.so"
for rep in 1 2 3; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/c2_new_$rep.json 2> $O/err || exit 1
  timeout -k 10 120 env $AB python -u bench.py --no-cpu-baseline > $O/c2_ab_$rep.json 2> $O/err || exit 1
done
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt60000 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 50 > $O/kt60000.json 2> $O/kt60000.err && \
cd $R && python3 profiles/kstats_live.py $O/kt60000/run_kernel_trace.csv --out $O/kt60000_live.csv > /dev/null
echo "rc=$?"
