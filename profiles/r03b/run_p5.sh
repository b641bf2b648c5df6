# device timeline of graph-replayed S-LBFGS epochs (is hipGraphLaunch's 20 ms of host time overlapped with
# the device, or in front of it?)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03p5
mkdir -p $O
cd /tmp
LBF_HOST_TIMING=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/ktg -o run -- python3 $R/bench.py --solver slbfgs --steps 2 --warmup 2 --no-cpu-baseline > $O/ktg.json 2> $O/ktg.err
echo "rc=$?"
