# Round 3, run K: forward split-K slabs reduced inside the GEMM launch (GemmDesc::fin_cnt) — bitwise test
# against fwd_reduce_act, the S-LBFGS / parity suites, cfg-4 bench: {anchor precompute, twin} x {fin, no fin}.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03k
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/ -q -x -m gpu --timeout 120 --timeout-method thread -k "split_k or slbfgs or batch_grads or loss_grad or fd_hvp or hvp" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp
for v in pre_fin twin_fin twin_nofin pre_nofin; do
  case $v in pre_fin) E="LBF_SLBFGS_ANCHOR=1 LBF_FWD_FIN=1";; twin_fin) E="LBF_SLBFGS_ANCHOR=0 LBF_FWD_FIN=1";;
             twin_nofin) E="LBF_SLBFGS_ANCHOR=0 LBF_FWD_FIN=0";; pre_nofin) E="LBF_SLBFGS_ANCHOR=1 LBF_FWD_FIN=0";; esac
  env $E timeout -k 10 200 python3 $R/bench.py --solver slbfgs --steps 4 --warmup 2 --no-cpu-baseline > $O/cfg4_$v.json 2> $O/cfg4_$v.err || exit 1
done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --steps 2 --warmup 1 --no-cpu-baseline > $O/kt4.json 2> $O/kt4.err || exit 1
cd $R
python3 profiles/kstats_live.py $O/kt4/run_kernel_trace.csv --out $O/kt4_live.csv
python3 profiles/gaps.py $O/kt4/run_kernel_trace.csv --top 12 > $O/gaps4.txt
echo "rc=$?"
