# standalone head: W loads before the tile's, LDS-only barriers (phase stamps, head parity, cfg 4)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03p13
mkdir -p $O
cd $R
timeout -k 10 200 python -u profiles/ktrace_head.py > $O/head_phases_after.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "head or slbfgs or fullsize or configs or hvp" > $O/tests.log 2>&1 || { echo "failed"; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 8 --warmup 2 --no-cpu-baseline > $O/cfg4_a.json 2> $O/cfg4_a.err && \
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 8 --warmup 2 --no-cpu-baseline > $O/cfg4_b.json 2> $O/cfg4_b.err
echo "rc=$?"
