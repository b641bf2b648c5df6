#!/bin/bash
# PMC passes over the GEMM probe (one counter group per pass; no trace domains combined with --pmc).
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/gemm_pmc
mkdir -p $O
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS"; do
  i=$((i+1))
  NS=${NS:-60000} timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 $R/profiles/gemm_probe.py > $O/p$i.log 2>&1
done
python3 - <<'PY'
import csv, glob, os, collections
O = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "gpurun_out", "gemm_pmc")
agg = collections.defaultdict(list)
for f in glob.glob(O + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "gemm_kernel" not in k and "head_kernel" not in k:
            continue
        agg[(k[:70], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:70s} {c:26s} n={len(v):3d} median={sorted(v)[len(v)//2]:.4g}")
PY
