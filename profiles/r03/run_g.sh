# Round 3, run G: dir_sweep with live-only history loads (S-LBFGS parity + cfg-4 dir vs LBF_DIR_FUSED=0);
# host-side timing of the speculative L-BFGS loop (enqueue vs wait per iteration) at 7500 and 60000 rows.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03g
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/ -q -x -m gpu --timeout 120 --timeout-method thread -k "slbfgs" > $O/slbfgs_tests.log 2>&1 || { echo "slbfgs tests failed"; tail -15 $O/slbfgs_tests.log; exit 1; }
tail -1 $O/slbfgs_tests.log
cd /tmp
for v in dir nodir; do
  case $v in dir) E="LBF_DIR_FUSED=1";; nodir) E="LBF_DIR_FUSED=0";; esac
  env $E timeout -k 10 200 python3 $R/bench.py --solver slbfgs --steps 4 --warmup 2 --no-cpu-baseline > $O/cfg4_$v.json 2> $O/cfg4_$v.err || exit 1
done
for n in 7500 60000; do
  LBF_HOST_TIMING=1 timeout -k 10 120 python3 $R/bench.py --samples $n --no-cpu-baseline > $O/bench_$n.json 2> $O/bench_$n.err || exit 1
done
echo "rc=$?"
