#!/bin/bash
# Round 6, run U: the Gram sweep's phase 1 without its duplicate operand loads (ga == ya, null gb / gc), against
# the previous commit's library (build_old/), interleaved on the two-loop microbenchmark, plus the parity files.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${RUN:-r06u}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
OLD=$R/lbfgs-ffnn_amd/build_old/liblbfgs_amd_abi3.so
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export LBF_LIB_PATH=$OLD; else unset LBF_LIB_PATH; fi
    timeout -k 10 240 python -u bench_two_loop.py --m 10,50 >> $O/two_loop_$v.jsonl 2>> $O/err.log || { echo "$v failed"; exit 1; }
  done
  echo "rep $rep done"
done
unset LBF_LIB_PATH
python3 - <<'PY'
import json, os
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/" + os.environ.get("RUN", "r06u")
for v in ("old", "new"):
    tl = [json.loads(l) for l in open(f"{O}/two_loop_{v}.jsonl")]
    for m in (10, 50):
        r = [t for t in tl if t["m"] == m]
        print(v, m, "frac", [t["roofline"]["frac"] for t in r], "gram", [t["gram_GBs"] for t in r], "coef", [t["hist_coef_us"] for t in r])
PY
echo "run u ok"
