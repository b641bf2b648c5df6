# Round 2, run AE: S-LBFGS FD pair of a Hessian step on the twin, pushed after the next step's evaluation: full GPU suite, cfg-4 A/B (build/ab = previous commit) x3, cfg-4 kernel trace.

export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02ae
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
AB="LBF_LIB_PATH=$R/lbfgs-ffnn_amd/build/ab/liblbfgs_amd.so"
for rep in 1 2 3; do
  timeout -k 10 300 python -u bench.py --solver slbfgs --steps 6 --warmup 1 --no-cpu-baseline > $O/c4_new_$rep.json 2> $O/err || exit 1
  timeout -k 10 300 env $AB python -u bench.py --solver slbfgs --steps 6 --warmup 1 --no-cpu-baseline > $O/c4_ab_$rep.json 2> $O/err || exit 1
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4 -o run -- python3 $R/bench.py --solver slbfgs --steps 3 --warmup 1 --no-cpu-baseline > $O/kt4.json 2> $O/kt4.err && \
cd $R && python3 profiles/kstats_live.py $O/kt4/run_kernel_trace.csv --out $O/kt4_live.csv > /dev/null || exit 1
echo "rc=$?"
echo "rc=$?"
