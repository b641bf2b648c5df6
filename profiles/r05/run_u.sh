#!/bin/bash
# round 5, run U: the driver's 8-rank bench command rehearsed on one GPU (eight RCCL processes over sockets):
# L-BFGS (the headline line) and S-LBFGS replicated; then the final suite on the tree after run T's revert.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05u
mkdir -p $O
cd $R
timeout -k 10 700 python -u profiles/r05/rehearse_ranks.py 8 --steps 10 --warmup 2 --no-cpu-baseline --device-warmup 0 > $O/rehearse8_lbfgs.txt 2>&1; echo "8-rank lbfgs rc $?"; tail -3 $O/rehearse8_lbfgs.txt
timeout -k 10 700 python -u profiles/r05/rehearse_ranks.py 8 --solver slbfgs --steps 2 --warmup 1 --no-cpu-baseline > $O/rehearse8_slbfgs.txt 2>&1; echo "8-rank slbfgs rc $?"; tail -3 $O/rehearse8_slbfgs.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; echo "suite rc $?"; tail -3 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc $?"; tail -1 $O/smoke.log
echo "run u ok"
