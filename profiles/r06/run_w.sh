#!/bin/bash
# Round 6, run W: dir_sweep's deferred split-K gradient with two rounds of split loads in flight per stripe (one
# round trip per 8 splits instead of 4), against the previous commit's library (build_old/): the whole -m gpu suite,
# the cfg-4 plan, then cfg 4 interleaved and rocprof kernel durations of both.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${RUN:-r06w}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|Error" $O/gpu_tests.log | head; tail -3 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
LBF_SHOW_PLAN=1 timeout -k 10 120 python -u bench.py --solver slbfgs --steps 1 --warmup 0 --no-cpu-baseline > $O/plan.json 2> $O/plan.err || { echo "plan failed"; exit 1; }
grep "lbf plan" $O/plan.err | sort | uniq -c | head -20
OLD=$R/lbfgs-ffnn_amd/build_old/liblbfgs_amd_abi3.so
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export LBF_LIB_PATH=$OLD; else unset LBF_LIB_PATH; fi
    timeout -k 10 240 python -u bench.py --solver slbfgs --steps 6 --no-cpu-baseline >> $O/cfg4_$v.jsonl 2>> $O/err.log || { echo "cfg4 $v failed"; exit 1; }
  done
done
for v in old new; do
  if [ $v = old ]; then export LBF_LIB_PATH=$OLD; else unset LBF_LIB_PATH; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4_$v -o run -- python3 bench.py --solver slbfgs --no-cpu-baseline --steps 3 --warmup 1 > $O/kt4_$v.json 2>> $O/err.log || { echo "prof $v failed"; exit 1; }
done
unset LBF_LIB_PATH
python3 - <<'PY'
import csv, glob, os, json
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/" + os.environ.get("RUN", "r06w")
for v in ("old", "new"):
    b = [json.loads(l)["value"] for l in open(f"{O}/cfg4_{v}.jsonl")]
    print(v, "cfg4", b)
    f = glob.glob(f"{O}/kt4_{v}/**/*kernel_stats.csv", recursive=True)[0]
    for row in csv.DictReader(open(f)):
        if "dir_" in row["Name"]:
            print("   ", row["Name"][:70], row["Calls"], round(float(row["AverageNs"]) / 1e3, 2))
PY
echo "run w ok"
