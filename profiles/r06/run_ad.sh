#!/bin/bash
# Round 6, run AD: the host-finished Wolfe trial with its backward and fused tail right behind the loss (no host round trip) (decision, pair push and
# the next direction on the device, so the next iteration speculates on the fused route at once), against the
# previous commit's library (build_old/): the whole -m gpu suite, then the driver shape and 400 iterations of cfg 2
# interleaved, and the per-iteration record times around rejections.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${RUN:-r06ad}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|Error" $O/gpu_tests.log | head; tail -3 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
OLD=$R/lbfgs-ffnn_amd/build_old/liblbfgs_amd_abi3.so
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export LBF_LIB_PATH=$OLD; else unset LBF_LIB_PATH; fi
    timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/b20_$v.jsonl 2>> $O/err.log || { echo "b20 $v failed"; exit 1; }
    timeout -k 10 240 python -u bench.py --steps 400 --no-cpu-baseline >> $O/b400_$v.jsonl 2>> $O/err.log || { echo "b400 $v failed"; exit 1; }
  done
done
for v in old new; do
  if [ $v = old ]; then export LBF_LIB_PATH=$OLD; else unset LBF_LIB_PATH; fi
  timeout -k 10 200 python -u profiles/r06/rej_cost.py > $O/rej_$v.txt 2>> $O/err.log || { echo "rej $v failed"; exit 1; }
done
unset LBF_LIB_PATH
python3 - <<'PY'
import json, os
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/" + os.environ.get("RUN", "r06ad")
for v in ("old", "new"):
    b20 = [json.loads(l) for l in open(f"{O}/b20_{v}.jsonl")]
    b4 = [json.loads(l) for l in open(f"{O}/b400_{v}.jsonl")]
    print(v, "b20", [d["value"] for d in b20], "evals/iter", [d["evals_per_iter"] for d in b20])
    print(v, "b400", [d["value"] for d in b4])
    print(open(f"{O}/rej_{v}.txt").read().split("first 30")[0])
PY
echo "run ab ok"
