"""Per-kernel medians of rocprofv3 --pmc passes (counter_collection.csv under the given dirs), with the
derived numbers the roofline uses:
  MFMA busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES * 4)   (4 SIMDs per CU... reported raw too)
  effective clock    = GRBM_GUI_ACTIVE / 8 / kernel time (MI355X_MICROARCH.md 'DVFS give-back')
  HBM bytes          = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (gfx950 FETCH_SIZE reads half of a wide stream)
    python3 pmc_summary.py DIR [DIR ...] [--match SUBSTR ...] > summary.txt
"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+")
ap.add_argument("--match", nargs="*", default=[])
ap.add_argument("--json", default=None)
a = ap.parse_args()
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in a.dirs:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if a.match and not any(m in k for m in a.match):
                continue
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, cs in sorted(agg.items()):
    row = {c: dict(n=len(v), median=statistics.median(v)) for c, v in sorted(cs.items())}
    if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
        row["hbm_bytes_median"] = 2 * row["FETCH_SIZE"]["median"] * 1024 + row["WRITE_SIZE"]["median"] * 1024
    out[k] = row
    print(k[:110])
    for c, v in row.items():
        print(f"    {c:28s} {v if not isinstance(v, dict) else v}")
if a.json:
    json.dump(out, open(a.json, "w"), indent=1)
