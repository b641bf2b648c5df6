#!/bin/bash
# Round 6, run R: rocprofv3 kernel durations of the history-step kernels, previous commit's library (build_old/)
# against the tree's, alternating: the 7500-row shard (tail_cols_fin), two-loop m = 10 (dir_cols_fin) and m = 50
# (fold_rows + hist_step).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${RUN:-r06r}
mkdir -p $O
cd $R
OLD=$R/lbfgs-ffnn_amd/build_old/liblbfgs_amd_abi3.so
for rep in 1 2; do
  for v in old new; do
    mkdir -p $O/${v}$rep
    if [ $v = old ]; then export LBF_LIB_PATH=$OLD; else unset LBF_LIB_PATH; fi
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}$rep/k7500 -o run -- python3 bench.py --samples 7500 --steps 400 --no-cpu-baseline > $O/${v}$rep/b7500.json 2> $O/err_${v}$rep.log || { echo "7500 $v failed"; exit 1; }
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}$rep/k2l -o run -- python3 bench_two_loop.py --m 10,50 > $O/${v}$rep/two_loop.jsonl 2>> $O/err_${v}$rep.log || { echo "two_loop $v failed"; exit 1; }
    echo "rep $rep $v done"
  done
done
unset LBF_LIB_PATH
python3 - <<'PY'
import csv, glob, os, json
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/" + os.environ.get("RUN", "r06r")
keys = ["tail_cols_fin", "tail_reduce", "dir_cols_fin", "hist_step", "fold_rows", "combine_small", "gemm_glds"]
for d in sorted(glob.glob(O + "/*[12]")):
    out = {}
    for sub in ("k7500", "k2l"):
        f = glob.glob(f"{d}/{sub}/**/*kernel_stats.csv", recursive=True)
        if not f:
            continue
        for row in csv.DictReader(open(f[0])):
            for k in keys:
                if k in row["Name"]:
                    out[f"{sub}:{row['Name'][:60]}"] = (int(row["Calls"]), round(float(row["AverageNs"]) / 1e3, 2))
    tl = [json.loads(l) for l in open(f"{d}/two_loop.jsonl")]
    b = json.loads(open(f"{d}/b7500.json").read().strip().splitlines()[-1])
    print(os.path.basename(d), "b7500", b["value"], "two_loop", [(t["m"], t["roofline"]["frac"], t["hist_coef_us"]) for t in tl])
    for k_, v_ in sorted(out.items()):
        print("   ", k_, v_)
PY
echo "run r ok"
