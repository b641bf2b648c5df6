"""Turn rocprofv3 PMC passes into per-launch HBM traffic for the bench's dominant kernel.

Run on the GPU box (two SEPARATE passes — FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950):
    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py ...
    python3 profiles/collect_pmc.py gpurun_out/pmc_fetch gpurun_out/pmc_write --section gemm_fwd[0] \
        --kernel "gemm_kernel<2, 2, 2, 2, true, false, 0, false>" --config 784,128,10:60000:1

Correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) reads half of the bytes of a wide coalesced
streaming read on gfx950, so bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.
"""
import argparse
import csv
import glob
import json
import os
import statistics


def per_dispatch(d, counter, kernel, largest_grid=False):
    """Counter values of every dispatch whose name contains `kernel`; largest_grid: only the dispatches with the
    largest grid among them (one instantiation serves several layers: e.g. cfg 5's dW GEMMs of layers 0 and 1,
    whose largest grid is layer 0's)."""
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            if kernel not in r.get("Kernel_Name", ""):
                continue
            rows.append((int(float(r.get("Grid_Size", 0) or 0)), float(r["Counter_Value"])))
    if largest_grid and rows:
        gmax = max(g for g, _ in rows)
        rows = [x for x in rows if x[0] == gmax]
    return [v for _, v in rows]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--section", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--config", required=True)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "pmc_traffic.json"))
    ap.add_argument("--largest-grid", action="store_true")
    a = ap.parse_args()
    fetch = per_dispatch(a.fetch_dir, "FETCH_SIZE", a.kernel, a.largest_grid)
    write = per_dispatch(a.write_dir, "WRITE_SIZE", a.kernel, a.largest_grid)
    if not fetch or not write:
        raise SystemExit(f"no samples: fetch={len(fetch)} write={len(write)}")
    f_kib, w_kib = statistics.median(fetch), statistics.median(write)
    out = dict(section=a.section, kernel=a.kernel, config=a.config, dispatches=[len(fetch), len(write)],
               fetch_kib_median=f_kib, write_kib_median=w_kib,
               hbm_bytes_per_launch=2 * f_kib * 1024 + w_kib * 1024,
               correction="bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE under-reads wide streams 2x)")
    # the file holds one entry per (section, config): replace this one's, keep the others
    entries = []
    if os.path.exists(a.out):
        try:
            old = json.load(open(a.out))
            entries = [e for e in (old if isinstance(old, list) else [old])
                       if (e.get("section"), e.get("config")) != (a.section, a.config)]
        except Exception:
            entries = []
    entries.append(out)
    json.dump(entries if len(entries) > 1 else out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
