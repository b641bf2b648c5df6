# Split-bf16 GEMM A/B: accuracy vs the oracle and cfg-2 / shard / cfg-3 benches per mode.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02split
mkdir -p $O
cd $R
timeout -k 10 300 python -u profiles/r02/split_ab.py > $O/accuracy.log 2>&1 && \
for m in 0 6 9; do
  LBF_GEMM_SPLIT=$m timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/bench_s$m.json 2> $O/bench_s$m.err || exit 1
  LBF_GEMM_SPLIT=$m timeout -k 10 120 python -u bench.py --samples 7500 --no-cpu-baseline > $O/bench7500_s$m.json 2> $O/bench7500_s$m.err || exit 1
  LBF_GEMM_SPLIT=$m timeout -k 10 120 python -u bench.py --dims 784,128,64,10 --acts relu,relu,linear --m 20 --no-cpu-baseline > $O/bench_cfg3_s$m.json 2> $O/bench_cfg3_s$m.err || exit 1
done
echo "rc=$?"
