# Round 2, run N: 64 x 128 forward tiles at the full 60000 rows too (build/t64: the tile rule's bound raised
# to four workgroups per CU) against the committed rule (128 x 128 there), interleaved.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02n
mkdir -p $O
cd $R
T64=$R/lbfgs-ffnn_amd/build/t64/liblbfgs_amd.so
NEW=$R/lbfgs-ffnn_amd/build/liblbfgs_amd.so
for rep in 1 2 3; do
  for v in new t64; do
    L=$NEW; [ $v = t64 ] && L=$T64
    LBF_LIB_PATH=$L timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 300 > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.err || exit 1
  done
done
LBF_LIB_PATH=$T64 timeout -k 10 120 python -u bench.py --samples 40000 --no-cpu-baseline > $O/b40000_t64.json 2> $O/b40000_t64.err || exit 1
LBF_LIB_PATH=$NEW timeout -k 10 120 python -u bench.py --samples 40000 --no-cpu-baseline > $O/b40000_new.json 2> $O/b40000_new.err || exit 1
echo "rc=0"
