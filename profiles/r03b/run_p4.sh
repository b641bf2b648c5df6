# where the S-LBFGS inner step's host enqueue time goes (eager epochs)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03p4
mkdir -p $O
cd $R
LBF_HOST_TIMING=2 LBF_SLBFGS_GRAPH=0 timeout -k 10 200 python -u bench.py --solver slbfgs --steps 3 --warmup 2 --no-cpu-baseline > $O/cfg4_ht2.json 2> $O/cfg4_ht2.err
echo "rc=$?"
