# Round 2, run AF: history step reads up to three staging rounds of Gram partial rows itself (no fold launch);
# S-LBFGS with 4096-element Gram chunks (131 workgroups at n = 535,818: no fold) vs the default chunk and
# build/ab (previous commit): full GPU suite, cfg 4 x3 each.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02af
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
AB="LBF_LIB_PATH=$R/lbfgs-ffnn_amd/build/ab/liblbfgs_amd.so"
for rep in 1 2 3; do
  timeout -k 10 300 env LBF_GRAM_CHUNK=4096 python -u bench.py --solver slbfgs --steps 6 --warmup 1 --no-cpu-baseline > $O/c4_c4096_$rep.json 2> $O/err || exit 1
  timeout -k 10 300 python -u bench.py --solver slbfgs --steps 6 --warmup 1 --no-cpu-baseline > $O/c4_new_$rep.json 2> $O/err || exit 1
  timeout -k 10 300 env $AB python -u bench.py --solver slbfgs --steps 6 --warmup 1 --no-cpu-baseline > $O/c4_ab_$rep.json 2> $O/err || exit 1
done
echo "rc=$?"
