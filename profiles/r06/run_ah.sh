#!/bin/bash
# Round 6, run AH: the speculative trial's Armijo test in its first backward GEMM (EarlyLs, gemm.hip
# gemm_early_exit; a first trial that fails sufficient decrease skips its backward and tail). The whole -m gpu
# suite (incl. test_early_armijo_exit_bitwise), smoke, then cfg 2 in the driver's shape, 400 iterations and the
# 7500-row shard, interleaved with the test left to the tail (LBF_NO_EARLY=1, same library).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${RUN:-r06ah}
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x -rf -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|Error|early" $O/tests.log | head; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
grep "rejected early" $O/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 $O/smoke.log
for rep in 1 2 3; do
  for v in off on; do
    if [ $v = off ]; then export LBF_NO_EARLY=1; else unset LBF_NO_EARLY; fi
    timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $O/b20_$v.jsonl 2>> $O/err.log || { echo "b20 $v failed"; exit 1; }
    timeout -k 10 240 python -u bench.py --steps 400 --no-cpu-baseline >> $O/b400_$v.jsonl 2>> $O/err.log || { echo "b400 $v failed"; exit 1; }
    timeout -k 10 240 python -u bench.py --steps 400 --samples 7500 --no-cpu-baseline >> $O/b7500_$v.jsonl 2>> $O/err.log || { echo "b7500 $v failed"; exit 1; }
  done
done
unset LBF_NO_EARLY
python3 - <<'PY'
import json, os
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/" + os.environ.get("RUN", "r06ah")
for b in ("b20", "b400", "b7500"):
    for v in ("off", "on"):
        L = [json.loads(l) for l in open(f"{O}/{b}_{v}.jsonl")]
        print(b, v, [d["value"] for d in L], "evals/iter", [d.get("evals_per_iter") for d in L],
              "loss-only/iter", [d.get("loss_only_trials_per_iter") for d in L])
PY
echo "run ah ok"
