#!/bin/bash
# Round 6, run AF: tail_reduce issuing the operand loads and the first round of 8 slab loads with the ring
# header (one round trip fewer before its sums), against the previous commit's library
# (build_old/): the whole -m gpu suite, then cfg 2 (400 iterations) and the 7500-row shard interleaved, rocprof of both.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${RUN:-r06af}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|Error" $O/tests.log | head; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
OLD=$R/lbfgs-ffnn_amd/build_old/liblbfgs_amd_abi3.so
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export LBF_LIB_PATH=$OLD; else unset LBF_LIB_PATH; fi
    timeout -k 10 240 python -u bench.py --steps 400 --no-cpu-baseline >> $O/b400_$v.jsonl 2>> $O/err.log || { echo "b400 $v failed"; exit 1; }
    timeout -k 10 240 python -u bench.py --steps 400 --samples 7500 --no-cpu-baseline >> $O/b7500_$v.jsonl 2>> $O/err.log || { echo "b7500 $v failed"; exit 1; }
  done
done
for v in old new; do
  if [ $v = old ]; then export LBF_LIB_PATH=$OLD; else unset LBF_LIB_PATH; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python3 bench.py --samples 7500 --steps 400 --no-cpu-baseline > $O/kt_$v.json 2>> $O/err.log || { echo "prof $v failed"; exit 1; }
done
unset LBF_LIB_PATH
python3 - <<'PY'
import csv, glob, os, json
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/" + os.environ.get("RUN", "r06af")
for v in ("old", "new"):
    b4 = [json.loads(l)["value"] for l in open(f"{O}/b400_{v}.jsonl")]
    b7 = [json.loads(l)["value"] for l in open(f"{O}/b7500_{v}.jsonl")]
    print(v, "b400", b4, "b7500", b7)
    f = glob.glob(f"{O}/kt_{v}/**/*kernel_stats.csv", recursive=True)[0]
    for row in csv.DictReader(open(f)):
        if "combine" in row["Name"] or "tail" in row["Name"]:
            print("   ", row["Name"][:70], row["Calls"], round(float(row["AverageNs"]) / 1e3, 2))
PY
echo "run z ok"
