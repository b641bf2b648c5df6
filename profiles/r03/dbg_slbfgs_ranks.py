"""Debug: S-LBFGS at world 2 with b = 1 (a rank's minibatch slice is empty): are the ranks bitwise equal,
with / without the twin stream and the two-launch history update?"""
import os
import sys
import threading

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

pkg = __graft_entry__.load_package()
dims, acts = [784, 16, 10], ["relu", "linear"]


def run(world, N, env, **kw):
    for k, v in env.items():
        os.environ[k] = v
    Xh, Yh = pkg.synth_mnist(N)
    X, Y = torch.from_numpy(Xh).cuda(), torch.from_numpy(Yh).cuda()
    ctxs = [pkg.Context(0, use_torch_stream=False) for _ in range(world)]
    if world > 1:
        pkg.Context.comm_init_local(ctxs)
    P0 = pkg.Mlp(ctxs[0], dims, acts).init_params(123, "cpu")
    torch.cuda.synchronize()
    out = [None] * world

    def th(r):
        net = pkg.Mlp(ctxs[r], dims, acts)
        P = P0.clone()
        h, _ = pkg.slbfgs_solve(net, P, X, Y, step=0.02, tol=0.0, lam=1e-4, pair_trace=64, **kw)
        torch.cuda.synchronize()
        out[r] = (h, P.double().cpu().numpy())

    ts = [threading.Thread(target=th, args=(r,)) for r in range(world)]
    [t.start() for t in ts]
    [t.join(120) for t in ts]
    return out


for env in [{}, {"LBF_SLBFGS_TWIN": "0"}, {"LBF_DIR_FUSED": "0"}, {"LBF_SLBFGS_TWIN": "0", "LBF_DIR_FUSED": "0"}]:
    for b, bh, N, ep in [(1, 1, 64, 1), (2, 2, 64, 1), (32, 16, 512, 1)]:
        os.environ.pop("LBF_SLBFGS_TWIN", None)
        os.environ.pop("LBF_DIR_FUSED", None)
        kw = dict(M=5, L=4, b=b, b_H=bh, max_epochs=ep)
        single = run(1, N, env, **kw)[0]
        res = run(2, N, env, **kw)
        d01 = np.abs(res[0][1] - res[1][1]).max()
        ds = np.abs(res[0][1] - single[1]).max() / np.abs(single[1]).max()
        print(f"{str(env):50s} b={b:2d} N={N}: rank0-rank1 max|dP| {d01:.3e}  rank0-single rel {ds:.3e} "
              f"loss {res[0][0]['loss']} {res[1][0]['loss']} single {single[0]['loss']}", flush=True)
        if d01 > 0:
            p0, p1 = res[0][0]["pairs"], res[1][0]["pairs"]
            for i in range(min(len(p0), len(p1), 8)):
                print("   pair", i, p0[i][:7], p1[i][:7])
