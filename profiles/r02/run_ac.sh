# Round 2, run AC: S-LBFGS Gram-sweep chunk per workgroup (LBF_GRAM_CHUNK: 1024 default -> 524 workgroups
# + a fold launch at n = 535,818; 4096 -> 131; 8192 -> 66), cfg 4 x2 each.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02ac
mkdir -p $O
cd $R
for rep in 1 2; do
  for c in 1024 2048 4096 8192; do
    timeout -k 10 300 env LBF_GRAM_CHUNK=$c python -u bench.py --solver slbfgs --steps 6 --warmup 1 --no-cpu-baseline > $O/c4_chunk${c}_$rep.json 2> $O/err || exit 1
  done
done
echo "rc=$?"
