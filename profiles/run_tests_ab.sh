# GPU tests, then the on-box A/B (run_ab.sh).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $R/gpurun_out/gpu_tests.log 2>&1 && \
bash $R/profiles/run_ab.sh
