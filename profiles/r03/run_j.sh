# Round 3, run J: S-LBFGS anchor gradients of the whole epoch up front (Mlp::batch_grads; no twin per step):
# S-LBFGS parity tests, cfg-4 bench anchor-precompute vs the twin (LBF_SLBFGS_ANCHOR=0), kernel trace.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03j
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/ -q -x -m gpu --timeout 120 --timeout-method thread -k "slbfgs or batch_grads" > $O/slbfgs_tests.log 2>&1 || { echo "slbfgs tests failed"; tail -30 $O/slbfgs_tests.log; exit 1; }
tail -1 $O/slbfgs_tests.log
cd /tmp
for v in pre twin; do
  case $v in pre) E="LBF_SLBFGS_ANCHOR=1";; twin) E="LBF_SLBFGS_ANCHOR=0";; esac
  env $E timeout -k 10 200 python3 $R/bench.py --solver slbfgs --steps 4 --warmup 2 --no-cpu-baseline > $O/cfg4_$v.json 2> $O/cfg4_$v.err || exit 1
done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --steps 2 --warmup 1 --no-cpu-baseline > $O/kt4.json 2> $O/kt4.err || exit 1
cd $R
python3 profiles/kstats_live.py $O/kt4/run_kernel_trace.csv --out $O/kt4_live.csv
python3 profiles/gaps.py $O/kt4/run_kernel_trace.csv --top 12 > $O/gaps4.txt
echo "rc=$?"
