# in-launch combine of the S-LBFGS direction (dir_cols_fin + combine workers): S-LBFGS suites, then cfg 4 A/B
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03p7
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "slbfgs or dp or ranks or fullsize or configs or graph or combine" > $O/slbfgs_tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 6 --warmup 2 --no-cpu-baseline > $O/cfg4_comb.json 2> $O/cfg4_comb.err && \
LBF_DIR_COMBINE=0 timeout -k 10 200 python -u bench.py --solver slbfgs --steps 6 --warmup 2 --no-cpu-baseline > $O/cfg4_nocomb.json 2> $O/cfg4_nocomb.err && \
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 6 --warmup 2 --no-cpu-baseline > $O/cfg4_comb2.json 2> $O/cfg4_comb2.err
echo "rc=$?"
