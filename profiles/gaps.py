"""Idle gaps on the GPU timeline of a rocprofv3 kernel trace: for every kernel name, how long the device
sat idle (no kernel of this process running) right before that kernel started, over the last `--tail`
dispatches (the timed region). A large gap before one kernel means the host (or a wait) was late with it.

    python3 profiles/gaps.py gpurun_out/.../run_kernel_trace.csv [--tail 2000]
"""
import argparse
import csv
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    return n.replace("void ", "").replace("lbf::", "")[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--tail", type=int, default=2000)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    ev = ev[-a.tail:]
    gap = defaultdict(list)
    busy = 0
    end = ev[0][1]
    for s, e, n in ev[1:]:
        gap[n].append(max(0, s - end) / 1000.0)
        busy += e - max(s, end) if e > end else 0
        end = max(end, e)
    span = (ev[-1][1] - ev[0][0]) / 1000.0
    print(f"span {span:.1f} us over {len(ev)} dispatches, busy {busy / 1000.0:.1f} us ({busy / 10.0 / span:.1f} %)")
    for n, g in sorted(gap.items(), key=lambda kv: -sum(kv[1])):
        g2 = sorted(g)
        print(f"{n:72s} n={len(g):5d} gap avg {sum(g) / len(g):7.2f} med {g2[len(g2) // 2]:7.2f} total {sum(g):9.1f} us")


if __name__ == "__main__":
    main()
