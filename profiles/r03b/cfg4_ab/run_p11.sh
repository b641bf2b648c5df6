# cfg 4 route A/B now that the epoch is device-bound (twin thread + free twin): in-launch forward split-K
# reduction, epoch-wide anchor precompute, 256-column direction sweep blocks
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03p11
mkdir -p $O
cd $R
B() { n=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --solver slbfgs --steps 8 --warmup 2 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { echo "$n failed"; exit 1; }; }
B base LBF_X=0 && B fwdfin LBF_FWD_FIN=1 && B anchor LBF_SLBFGS_ANCHOR=1 && B dircols256 LBF_DIR_COLS=256 && B base2 LBF_X=0 && B fwdfin2 LBF_FWD_FIN=1
echo "rc=$?"
