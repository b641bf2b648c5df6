# Round 3, run O: the direct-operand GEMM's intermittent NaN (784-16-10): stress with 3 register sets
# (refill right behind the MFMAs that read the set) vs 4 (refilled one k-tile later).
R=$GRAFT_REPO_ROOT
cd $R
for v in 4 3 4; do
  LBF_GEMM_DIRECT_SETS=$v timeout -k 10 200 python3 profiles/r03/stress_direct.py > gpurun_out/stress_sets$v.log 2>&1 || exit 1
  echo "sets=$v"; tail -2 gpurun_out/stress_sets$v.log
done
