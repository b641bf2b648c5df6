# End-of-round evidence: GPU tests, the bench lines and kernel traces (run_final.sh), PMC traffic.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
bash $R/profiles/run_pmc.sh > $O/pmc.log 2>&1 && grep -q "rc=0" $O/pmc.log && \
cp $O/pmc_traffic.json $R/profiles/pmc_traffic.json && \
bash $R/profiles/run_final.sh > $O/final.log 2>&1 && grep -q "rc=0" $O/final.log
echo "rc=$?"
