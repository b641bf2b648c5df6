# Round 2, run Y: software-pipelined head tile (dW rounds and delta row strips) for 32/64-row GEMM tiles and
# the standalone head: full GPU suite, then A/B (build/ab = previous commit) at the 7500 / 15000-row shards,
# cfg 4 (S-LBFGS) and cfg 2, plus a kernel trace of the shard.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02y
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
AB="LBF_LIB_PATH=$R/lbfgs-ffnn_amd/build/ab/liblbfgs_amd.so"
for rep in 1 2; do
  timeout -k 10 120 python -u bench.py --samples 7500 --no-cpu-baseline > $O/s7500_new_$rep.json 2> $O/err || exit 1
  timeout -k 10 120 env $AB python -u bench.py --samples 7500 --no-cpu-baseline > $O/s7500_ab_$rep.json 2> $O/err || exit 1
  timeout -k 10 120 python -u bench.py --samples 15000 --no-cpu-baseline > $O/s15000_new_$rep.json 2> $O/err || exit 1
  timeout -k 10 120 env $AB python -u bench.py --samples 15000 --no-cpu-baseline > $O/s15000_ab_$rep.json 2> $O/err || exit 1
  timeout -k 10 300 python -u bench.py --solver slbfgs --steps 6 --warmup 1 --no-cpu-baseline > $O/c4_new_$rep.json 2> $O/err || exit 1
  timeout -k 10 300 env $AB python -u bench.py --solver slbfgs --steps 6 --warmup 1 --no-cpu-baseline > $O/c4_ab_$rep.json 2> $O/err || exit 1
done
timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/c2_new.json 2> $O/err || exit 1
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt7500 -o run -- python3 $R/bench.py --samples 7500 --no-cpu-baseline --steps 50 > $O/kt7500.json 2> $O/kt7500.err && \
cd $R && python3 profiles/kstats_live.py $O/kt7500/run_kernel_trace.csv --out $O/kt7500_live.csv > /dev/null
echo "rc=$?"
