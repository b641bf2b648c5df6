#!/bin/bash
# Round 6, run AC: the fused host-finished gradient extended to the Armijo search (CUDA semantics), against
# the previous commit's library (build_old/, which has it for Wolfe only): the whole -m gpu suite, then the deep
# config (Armijo, m = 10) and cfg 2 with the Armijo line search, interleaved.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${RUN:-r06ac}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|Error" $O/gpu_tests.log | head; tail -3 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
OLD=$R/lbfgs-ffnn_amd/build_old/liblbfgs_amd_abi3.so
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export LBF_LIB_PATH=$OLD; else unset LBF_LIB_PATH; fi
    timeout -k 10 240 python -u bench.py --dims 784,256,128,64,10 --acts relu,relu,relu,linear --line-search armijo --init cuda --steps 200 --no-cpu-baseline >> $O/deep_$v.jsonl 2>> $O/err.log || { echo "deep $v failed"; exit 1; }
    timeout -k 10 240 python -u bench.py --line-search armijo --init cuda --steps 400 --no-cpu-baseline >> $O/armijo_$v.jsonl 2>> $O/err.log || { echo "armijo $v failed"; exit 1; }
  done
done
unset LBF_LIB_PATH
python3 - <<'PY'
import json, os
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/" + os.environ.get("RUN", "r06ac")
for v in ("old", "new"):
    for k in ("deep", "armijo"):
        b = [json.loads(l) for l in open(f"{O}/{k}_{v}.jsonl")]
        print(v, k, [d["value"] for d in b], "evals/iter", [d["evals_per_iter"] for d in b])
PY
echo "run ac ok"
