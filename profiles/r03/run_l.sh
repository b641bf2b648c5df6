# Round 3, run L: full GPU suite on the committed tree; 7500-row shard A/B of the forward route (32x128
# EPI_HEAD tile vs split-K 128x128 + reduce + standalone head, with the reduce separate or in-launch).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03l
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/ -q -x -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
cd /tmp
for v in tile32 splitk splitk_fin; do
  case $v in tile32) E="LBF_FWD_TILE32=1";; splitk) E="LBF_FWD_TILE32=0";; splitk_fin) E="LBF_FWD_TILE32=0 LBF_FWD_FIN=1";; esac
  env $E timeout -k 10 120 python3 $R/bench.py --samples 7500 --no-cpu-baseline > $O/bench_7500_$v.json 2> $O/bench_7500_$v.err || exit 1
done
LBF_FWD_TILE32=0 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/kt7500_splitk -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500_splitk.json 2> $O/kt7500_splitk.err || exit 1
cd $R
python3 profiles/kstats_live.py --spec $O/kt7500_splitk/run_kernel_trace.csv --out $O/kt7500_splitk_live.csv
echo "rc=$?"
