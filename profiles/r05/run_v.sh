#!/bin/bash
# round 5, run V: the 8-rank S-LBFGS rehearsal after bench.py's fix (run U: the epoch's all-reduce won the
# breakdown at 8 ranks over sockets and was not sampled in the timed region -> KeyError); the one-GPU cfg-4 line.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05v
mkdir -p $O
cd $R
timeout -k 10 700 python -u profiles/r05/rehearse_ranks.py 8 --solver slbfgs --steps 2 --warmup 1 --no-cpu-baseline > $O/rehearse8_slbfgs.txt 2>&1; echo "8-rank slbfgs rc $?"; grep -v "^\[W\|Gloo\|amdgpu" $O/rehearse8_slbfgs.txt | tail -3
timeout -k 10 700 python -u profiles/r05/rehearse_ranks.py 4 --solver slbfgs --slbfgs-dp sliced --steps 2 --warmup 1 --no-cpu-baseline > $O/rehearse4_slbfgs_sliced.txt 2>&1; echo "4-rank sliced rc $?"; grep -v "^\[W\|Gloo\|amdgpu" $O/rehearse4_slbfgs_sliced.txt | tail -3
timeout -k 10 200 python -u bench.py --solver slbfgs --steps 6 --no-cpu-baseline > $O/cfg4.json 2> $O/cfg4.err; echo "cfg4 rc $?"; tail -1 $O/cfg4.json | cut -c1-400
echo "run v ok"
