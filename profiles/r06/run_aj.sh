#!/bin/bash
# Round 6, run AJ: cfg 4 (S-LBFGS, which never takes the early Armijo test) with the library before the early test
# (commit 4019130, build_old/) and the final one, interleaved: does the GEMM entry's extra argument test cost the
# latency-bound minibatch launches anything?
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${RUN:-r06aj}
mkdir -p $O
cd $R
OLD=$R/lbfgs-ffnn_amd/build_old/liblbfgs_amd_abi3.so
test -f $OLD || { echo "no old library"; exit 1; }
for rep in 1 2 3 4; do
  for v in old new; do
    if [ $v = old ]; then export LBF_LIB_PATH=$OLD; else unset LBF_LIB_PATH; fi
    timeout -k 10 240 python -u bench.py --solver slbfgs --steps 6 --no-cpu-baseline >> $O/cfg4_$v.jsonl 2>> $O/err.log || { echo "cfg4 $v failed"; exit 1; }
  done
done
unset LBF_LIB_PATH
python3 - <<'PY'
import json, os
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/" + os.environ.get("RUN", "r06aj")
for v in ("old", "new"):
    print(v, [json.loads(l)["value"] for l in open(f"{O}/cfg4_{v}.jsonl")])
PY
echo "run aj ok"
