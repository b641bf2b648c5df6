"""Cost of a rejected speculative trial at cfg 2 (784-128-10, N = 60000, Wolfe, m = 10): per-iteration host
record times of a 400-iteration run, split by line-search trials (1 = the speculative first trial accepted)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402


def main():
    pkg = __graft_entry__.load_package()
    ctx = pkg.Context(0)
    Xh, Yh = pkg.synth_mnist(60000)
    X, Y = torch.from_numpy(Xh).cuda(), torch.from_numpy(Yh).cuda()
    net = pkg.Mlp(ctx, [784, 128, 10], ["relu", "linear"])
    P = net.init_params(123, "cpu")
    run = pkg.LbfgsRun(net, P, X, Y, m=10, max_iters=1 << 20, tol=0.0, record_cap=600)
    run.iterate(25)
    torch.cuda.synchronize()
    n0 = run.hist.size
    run.iterate(int(os.environ.get("REJ_ITERS", "400")))
    torch.cuda.synchronize()
    d = run.hist.as_dict()
    t = d["time_ms"][n0 - 1:]
    dt = np.diff(t) * 1e3
    tr = d["ls_trials"][n0:]
    print("iterations", len(dt), "mean us", dt.mean().round(1))
    for k in sorted(set(tr.tolist())):
        sel = dt[tr == k]
        print(f"ls_trials {k}: {len(sel)} iterations, median {np.median(sel):.1f} us, mean {sel.mean():.1f} us")
    # the iteration after a rejection (the speculative queue restarts)
    after = dt[1:][tr[:-1] > 1]
    if len(after):
        print(f"after a rejection: median {np.median(after):.1f} us, mean {after.mean():.1f} us")
    print("first 30 (trials, us):", [(int(a), round(float(b), 1)) for a, b in zip(tr[:30], dt[:30])])
    run.close()


if __name__ == "__main__":
    main()
