# Round 3, run D: host-side launch costs; the S-LBFGS rank-equality debug; rank / DP / S-LBFGS tests after the
# words-buffer fix (aborted speculative collectives); the first-pair HVP comparison; cfg 4 with the
# vectorised two-launch update (A/B) and host enqueue timing; cfg-4 kernel trace.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03d
mkdir -p $O
cd $R
timeout -k 10 90 ./profiles/micro/launch_floor > $O/launch_floor.txt 2>&1 || echo "launch_floor failed"
timeout -k 10 200 python -u profiles/r03/dbg_slbfgs_ranks.py > $O/dbg_slbfgs.log 2>&1 || { echo "dbg failed"; tail -5 $O/dbg_slbfgs.log; }
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "ranks or dp or slbfgs or cfg4 or armijo or spec" > $O/tests.log 2>&1
echo "tests rc=$?"; grep -E "FAILED|passed|failed" $O/tests.log | tail -8
timeout -k 10 200 python -u profiles/r03/diag_pair0.py > $O/diag_pair0.log 2>&1; echo "diag rc=$?"
LBF_HOST_TIMING=1 timeout -k 10 200 python -u bench.py --solver slbfgs --steps 6 --warmup 1 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err && \
LBF_HOST_TIMING=1 LBF_DIR_FUSED=0 timeout -k 10 200 python -u bench.py --solver slbfgs --steps 6 --warmup 1 --no-cpu-baseline > $O/bench_cfg4_nodir.json 2> $O/bench_cfg4_nodir.err && \
LBF_HOST_TIMING=1 LBF_SLBFGS_TWIN=0 timeout -k 10 200 python -u bench.py --solver slbfgs --steps 6 --warmup 1 --no-cpu-baseline > $O/bench_cfg4_notwin.json 2> $O/bench_cfg4_notwin.err && \
cd /tmp && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --steps 3 --warmup 1 --no-cpu-baseline > $O/kt4.json 2> $O/kt4.err && \
cd $R && python3 profiles/kstats_live.py $O/kt4/run_kernel_trace.csv --out $O/kt4_live.csv > /dev/null
echo "rc=$?"
