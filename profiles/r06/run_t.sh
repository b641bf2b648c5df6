#!/bin/bash
# Round 6, run T: nontemporal stores in the large-n history sweeps, interleaved A/B on the two-loop
# microbenchmark: base, LBF_GRAM_NTST=1 (the Gram sweep's s / y / g stores), LBF_COMB_NTST=1 (the combine's
# direction / trial stores), both.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${RUN:-r06t}
mkdir -p $O
cd $R
for rep in 1 2 3; do
  for v in base gram comb both; do
    case $v in base) E="";; gram) E="LBF_GRAM_NTST=1";; comb) E="LBF_COMB_NTST=1";; both) E="LBF_GRAM_NTST=1 LBF_COMB_NTST=1";; esac
    env $E timeout -k 10 240 python -u bench_two_loop.py --m 10,50 >> $O/two_loop_$v.jsonl 2>> $O/err.log || { echo "$v failed"; exit 1; }
  done
  echo "rep $rep done"
done
python3 - <<'PY'
import json, os
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/" + os.environ.get("RUN", "r06t")
for v in ("base", "gram", "comb", "both"):
    tl = [json.loads(l) for l in open(f"{O}/two_loop_{v}.jsonl")]
    for m in (10, 50):
        r = [t for t in tl if t["m"] == m]
        print(v, m, "frac", [t["roofline"]["frac"] for t in r], "gram", [t["gram_GBs"] for t in r], "comb", [t["combine_GBs"] for t in r])
PY
echo "run t ok"
