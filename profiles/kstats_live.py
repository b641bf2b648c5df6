"""Per-kernel statistics from a rocprofv3 --kernel-trace CSV, separating live launches from the
speculative ones that exit at their abort check (a few microseconds: the iteration chain after a
rejected line-search trial, see solvers.cpp iterate_spec).

    python3 profiles/kstats_live.py gpurun_out/prof/run_kernel_trace.csv [--min-us 5] [--out file.csv]

rocprofv3's own --stats average mixes both; bench.py's HIP-event average of the dominant kernel is
over sampled launches, which are almost all live, so compare it with avg_live_us here.
"""
import argparse
import collections
import csv
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--min-us", type=float, default=5.0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(a.trace)):
        d[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = []
    for name, v in d.items():
        live = [x for x in v if x > a.min_us]
        rows.append(dict(kernel=name, calls=len(v), live_calls=len(live),
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
