"""Inter-kernel gaps on one stream from a rocprofv3 --kernel-trace CSV: for each (kernel, next kernel) pair,
the median time from the first's end to the second's start (launch latency shows inside the durations; a
gap is extra idle time).   python3 profiles/gaps.py run_kernel_trace.csv [--top 8]"""
import argparse
import collections
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    by = collections.defaultdict(list)
    for r in rows:
        by[r["Stream_Id"]].append(r)
    for sid, v in sorted(by.items(), key=lambda kv: -len(kv[1])):
        if len(v) < 20:
            continue
        v.sort(key=lambda r: int(r["Start_Timestamp"]))
        gaps = collections.defaultdict(list)
        for x, y in zip(v[len(v) // 4:-1], v[len(v) // 4 + 1:]):
            g = (int(y["Start_Timestamp"]) - int(x["End_Timestamp"])) / 1e3
            if -1 < g < 200:
                gaps[(x["Kernel_Name"][:38], y["Kernel_Name"][:38])].append(g)
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in v[len(v) // 4:]) / 1e6
        span = (int(v[-1]["End_Timestamp"]) - int(v[len(v) // 4]["Start_Timestamp"])) / 1e6
        print(f"stream {sid}: {len(v)} launches, last 3/4: busy {busy:.2f} ms of {span:.2f} ms")
        for k, g in sorted(gaps.items(), key=lambda kv: -sum(kv[1]))[:a.top]:
            print(f"  {k[0]:38s} -> {k[1]:38s} n={len(g):5d} med={statistics.median(g):6.2f} sum={sum(g) / 1e3:7.2f} ms")


if __name__ == "__main__":
    main()
