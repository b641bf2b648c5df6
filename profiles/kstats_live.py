"""Per-kernel statistics from a rocprofv3 --kernel-trace CSV.

    python3 profiles/kstats_live.py gpurun_out/prof/run_kernel_trace.csv [--spec] [--out file.csv]

Without --spec every launch counts (S-LBFGS, GD, the host-driven L-BFGS: nothing is ever aborted).
With --spec (the speculative L-BFGS pipeline, solvers.cpp iterate_spec) the launches queued behind a
rejected line-search trial exit at their abort check; for each kernel such a launch is told apart by
its duration: below --abort-frac (default 0.25) of that kernel's median. The big GEMMs split cleanly
(aborted 3-5 us against 30-140 us live); for kernels whose live launches are themselves a few
microseconds the split is not attempted (fewer than --abort-frac x median means nothing there), so
their averages include the few aborted launches (reported in aborted_calls = 0 and calls). The
dropped counts are in the output, so nothing is filtered silently.

rocprofv3's own --stats average mixes both; bench.py's HIP-event average of the dominant kernel is
over sampled launches, which are almost all live, so compare it with avg_live_us here.
"""
import argparse
import collections
import csv
import statistics
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--spec", action="store_true", help="speculative L-BFGS trace: drop aborted launches")
    ap.add_argument("--abort-frac", type=float, default=0.25)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(a.trace)):
        d[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = []
    for name, v in d.items():
        cut = a.abort_frac * statistics.median(v) if a.spec else 0.0
        live = [x for x in v if x >= cut]
        rows.append(dict(kernel=name, calls=len(v), live_calls=len(live), aborted_calls=len(v) - len(live),
                         avg_live_us=round(sum(live) / len(live), 3) if live else 0.0,
                         min_live_us=round(min(live), 3) if live else 0.0,
                         max_live_us=round(max(live), 3) if live else 0.0,
                         total_us=round(sum(v), 1)))
    rows.sort(key=lambda r: -r["total_us"])
    tot = sum(r["total_us"] for r in rows)
    for r in rows:
        r["pct"] = round(100 * r["total_us"] / tot, 2)
    out = open(a.out, "w") if a.out else sys.stdout
    w = csv.DictWriter(out, fieldnames=list(rows[0].keys()))
    w.writeheader()
    w.writerows(rows)


if __name__ == "__main__":
    main()
