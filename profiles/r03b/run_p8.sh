# cfg-4 kernel trace with the twin thread: per-stream busy / gaps of the context stream
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03p8
mkdir -p $O
cd /tmp
LBF_HOST_TIMING=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --steps 2 --warmup 2 --no-cpu-baseline > $O/kt4.json 2> $O/kt4.err
cd $R
python3 profiles/gaps.py --top 30 $O/kt4/run_kernel_trace.csv > $O/gaps_cfg4.txt
echo "rc=$?"
