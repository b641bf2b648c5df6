# DP route on one GPU (1-rank RCCL communicator): parity tests, then the per-rank bench at the 8-rank
# shard size through the DP route (local reduce + ncclAllReduce + tail) vs the plain route.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py -x -v --timeout 120 --timeout-method thread > $O/gpu_dp.log 2>&1 && \
timeout -k 10 120 python -u bench.py --samples 7500 --no-cpu-baseline --steps 100 --comm1 > $O/bench_7500_comm1.json 2> $O/bench_7500_comm1.err && \
timeout -k 10 120 python -u bench.py --samples 7500 --no-cpu-baseline --steps 100 > $O/bench_7500.json 2> $O/bench_7500.err && \
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_7500c -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 --comm1 > $R/$O/prof_7500c.json 2> $R/$O/prof_7500c.err
echo "rc=$?"
