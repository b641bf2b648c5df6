"""Debug: cfg-2 Armijo trajectories through the single route, a 1-rank RCCL communicator, a 1-rank and a
2-rank in-process group, with and without speculation (LBF_SPEC_DEPTH=0 is read at solver creation)."""
import os
import sys
import threading

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

pkg = __graft_entry__.load_package()
dims, acts, N = [784, 128, 10], ["relu", "linear"], 60000
Xh, Yh = pkg.synth_mnist(N)
X, Y = torch.from_numpy(Xh).cuda(), torch.from_numpy(Yh).cuda()
ctx = pkg.Context(0)
P0 = pkg.Mlp(ctx, dims, acts).init_params(123, "cpu")
ITERS = 10


def show(name, h):
    print(f"{name:28s} loss {np.array2string(h['loss'][:ITERS], precision=6, max_line_width=250)}")
    print(f"{'':28s} trials {h['ls_trials'][:ITERS]} acc {h['accepted'][:ITERS]} "
          f"alpha {np.array2string(h['alpha'][:ITERS], precision=4, max_line_width=250)}", flush=True)


def run_world(world, spec):
    os.environ["LBF_SPEC_DEPTH"] = str(spec)
    ctxs = [pkg.Context(0, use_torch_stream=False) for _ in range(world)]
    pkg.Context.comm_init_local(ctxs)
    torch.cuda.synchronize()
    out = [None] * world
    Xs = [X[N * r // world: N * (r + 1) // world].contiguous() for r in range(world)]
    Ys = [Y[N * r // world: N * (r + 1) // world].contiguous() for r in range(world)]

    def th(r):
        net = pkg.Mlp(ctxs[r], dims, acts)
        P = P0.clone()
        out[r] = pkg.lbfgs_solve(net, P, Xs[r], Ys[r], n_global=N, line_search="armijo", m=10, max_iters=ITERS,
                                 tol=0.0)[0]
        torch.cuda.synchronize()

    ts = [threading.Thread(target=th, args=(r,)) for r in range(world)]
    [t.start() for t in ts]
    [t.join(120) for t in ts]
    return out[0]


for spec in (3, 0):
    os.environ["LBF_SPEC_DEPTH"] = str(spec)
    net = pkg.Mlp(ctx, dims, acts)
    show(f"single spec={spec}", pkg.lbfgs_solve(net, P0.clone(), X, Y, line_search="armijo", m=10, max_iters=ITERS,
                                                 tol=0.0)[0])
    c1 = pkg.Context(0)
    c1.comm_init(1, 0, pkg.Context.unique_id())
    net = pkg.Mlp(c1, dims, acts)
    show(f"rccl1 spec={spec}", pkg.lbfgs_solve(net, P0.clone(), X, Y, line_search="armijo", m=10, max_iters=ITERS,
                                                tol=0.0)[0])
    show(f"local1 spec={spec}", run_world(1, spec))
    show(f"local2 spec={spec}", run_world(2, spec))
