#!/bin/bash
# Round 6, run S: tail_reduce with every slab of a launch in one round (U = 24 loads per stripe when a launch
# has more than 32 splits) against three rounds of 8 (LBF_TAIL_WIDE=0): cfg 2 (82 slabs) interleaved, rocprof
# kernel durations of both, and the gradient-path tests.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${RUN:-r06s}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for v in 0 1; do
    LBF_TAIL_WIDE=$v timeout -k 10 240 python -u bench.py --steps 400 --no-cpu-baseline >> $O/b400_w$v.jsonl 2>> $O/err.log || { echo "b400 $v failed"; exit 1; }
  done
done
for v in 0 1; do
  LBF_TAIL_WIDE=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_w$v -o run -- python3 bench.py --steps 100 --no-cpu-baseline > $O/kt_w$v.json 2>> $O/err.log || { echo "prof $v failed"; exit 1; }
done
python3 - <<'PY'
import csv, glob, os, json
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/" + os.environ.get("RUN", "r06s")
for v in (0, 1):
    b = [json.loads(l)["value"] for l in open(f"{O}/b400_w{v}.jsonl")]
    print("wide", v, "b400", b)
    f = glob.glob(f"{O}/kt_w{v}/**/*kernel_stats.csv", recursive=True)[0]
    for row in csv.DictReader(open(f)):
        if "tail" in row["Name"] or "combine_small" in row["Name"]:
            print("   ", row["Name"][:70], row["Calls"], round(float(row["AverageNs"]) / 1e3, 2))
PY
echo "run s ok"
