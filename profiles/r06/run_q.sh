#!/bin/bash
# Round 6, run Q: the history step's staging by rows and its parallel evict shift (csrc/hist_core.hpp).
# The whole -m gpu suite on the new tree, its phase stamps, then an interleaved A/B against the previous
# commit's library (build_old/): two-loop m = 10 / 50, cfg 2 400 iterations, the 7500-row shard.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${RUN:-r06q}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|Error" $O/gpu_tests.log | head; tail -3 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 240 python -u profiles/r06/ktrace_hist.py --m 10,50 > $O/ktrace_hist.txt 2>&1 || { echo "ktrace failed"; tail -3 $O/ktrace_hist.txt; exit 1; }
grep "^m=" $O/ktrace_hist.txt
OLD=$R/lbfgs-ffnn_amd/build_old/liblbfgs_amd_abi3.so
for rep in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export LBF_LIB_PATH=$OLD; else unset LBF_LIB_PATH; fi
    timeout -k 10 240 python -u bench_two_loop.py --m 10,50 >> $O/two_loop_$v.jsonl 2>> $O/err.log || { echo "two_loop $v failed"; exit 1; }
    timeout -k 10 240 python -u bench.py --steps 400 --no-cpu-baseline >> $O/b400_$v.jsonl 2>> $O/err.log || { echo "b400 $v failed"; exit 1; }
    timeout -k 10 240 python -u bench.py --steps 400 --samples 7500 --no-cpu-baseline >> $O/b7500_$v.jsonl 2>> $O/err.log || { echo "b7500 $v failed"; exit 1; }
    echo "rep $rep $v done"
  done
done
unset LBF_LIB_PATH
python3 - <<'PY'
import json, glob, os
O = os.environ.get("GRAFT_REPO_ROOT", ".") + "/gpurun_out/" + os.environ.get("RUN", "r06q")
for v in ("old", "new"):
    tl = [json.loads(l) for l in open(f"{O}/two_loop_{v}.jsonl")]
    b4 = [json.loads(l)["value"] for l in open(f"{O}/b400_{v}.jsonl")]
    b7 = [json.loads(l)["value"] for l in open(f"{O}/b7500_{v}.jsonl")]
    print(v, "two_loop", [(d["m"], d["roofline"]["frac"], d["hist_coef_us"]) for d in tl], "b400", b4, "b7500", b7)
PY
echo "run q ok"
