# Round 3, run M: dir_sweep with 512 columns per block (one round of blocks at cfg 4's n) vs 256; the
# FD-HVP kink test; S-LBFGS suites.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03m
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/ -q -x -m gpu --timeout 120 --timeout-method thread -k "slbfgs or kink or two_loop or dir" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp
for v in c512 c256 c512b; do
  case $v in c512|c512b) E="LBF_DIR_COLS=512";; c256) E="LBF_DIR_COLS=256";; esac
  env $E timeout -k 10 200 python3 $R/bench.py --solver slbfgs --steps 4 --warmup 2 --no-cpu-baseline > $O/cfg4_$v.json 2> $O/cfg4_$v.err || exit 1
done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --steps 2 --warmup 1 --no-cpu-baseline > $O/kt4.json 2> $O/kt4.err || exit 1
cd $R
python3 profiles/kstats_live.py $O/kt4/run_kernel_trace.csv --out $O/kt4_live.csv
echo "rc=$?"
