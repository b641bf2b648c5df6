#!/bin/bash
# PMC passes over the bench for the small kernels (one counter group per pass).
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/small_pmc
mkdir -p $O
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 $R/bench.py --cpu-iters 0 --steps 20 --warmup 2 > $O/p$i.log 2>&1
done
python3 - <<'PY'
import csv, glob, os, collections
O = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "gpurun_out", "small_pmc")
agg = collections.defaultdict(list)
for f in glob.glob(O + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "gemm_kernel" in k:
            continue
        agg[(k.split("(")[0][-28:], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:28s} {c:22s} n={len(v):3d} median={sorted(v)[len(v)//2]:.4g}")
PY
