# A/B on one box: the committed library (build/ab) against the working tree's (build), interleaved
# benches plus a kernel trace of each (cfg 2 and the 7500-row shard).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab
mkdir -p $O
cd $R
AB=$R/lbfgs-ffnn_amd/build/ab/liblbfgs_amd.so
NEW=$R/lbfgs-ffnn_amd/build/liblbfgs_amd.so
ok=0
for rep in 1 2; do
  for v in ab new; do
    L=$AB; [ $v = new ] && L=$NEW
    LBF_LIB_PATH=$L timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 300 > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.err || { ok=1; break 2; }
    LBF_LIB_PATH=$L timeout -k 10 120 python -u bench.py --samples 7500 --no-cpu-baseline --steps 300 > $O/s_${v}_$rep.json 2> $O/s_${v}_$rep.err || { ok=1; break 2; }
  done
done
[ $ok = 0 ] && for v in ab new; do
  L=$AB; [ $v = new ] && L=$NEW
  (cd /tmp && LBF_LIB_PATH=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python3 $R/bench.py --no-cpu-baseline --steps 50 > $O/kt_$v.json 2> $O/kt_$v.err) || { ok=1; break; }
  python3 $R/profiles/kstats_live.py $O/kt_$v/run_kernel_trace.csv --out $O/kt_${v}_live.csv > /dev/null
done
echo "rc=$ok"
