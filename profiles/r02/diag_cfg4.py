"""Diagnostic: cfg-4 (784-512-256-10) loss/grad vs the oracle at full size and on gathered minibatches,
then device S-LBFGS epochs at a few steps."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

os.environ["LBF_SHOW_PLAN"] = "1"
pkg = __graft_entry__.load_package()
O = __graft_entry__.load_oracle()
dims, acts = [784, 512, 256, 10], ["relu", "relu", "linear"]
Xh, Yh = pkg.synth_mnist(60000)
X, Y = torch.from_numpy(Xh).cuda(), torch.from_numpy(Yh).cuda()
X64, Y64 = Xh.astype(np.float64), Yh.astype(np.float64)
ctx = pkg.Context(0)
onet = O.Net(dims, acts)
segs, off = [], 0
for l in range(3):
    i, o = dims[l], dims[l + 1]
    segs.append((f"W{l}", off, off + i * o))
    segs.append((f"b{l}", off + i * o, off + (i + 1) * o))
    off += (i + 1) * o
net = pkg.Mlp(ctx, dims, acts)
P = net.init_params(123, "cpu")
P64 = P.double().cpu().numpy()
for N, B in [(60000, None), (60000, 256), (60000, 128), (60000, 32), (7500, None)]:
    if B is None:
        l, g = net.loss_grad(P, X[:N], Y[:N], l2=1e-4)
        lr, gr = onet.loss_grad(P64, X64[:N], Y64[:N], lam=1e-4)
    else:
        rows = O.sample_indices(N, B, seed=7, calls=1)[0]
        idx = torch.from_numpy(rows.astype(np.int32)).cuda()
        l, g = net.loss_grad(P, X, Y, idx=idx, l2=1e-4)
        lr, gr = onet.loss_grad(P64, X64, Y64, idx=rows, lam=1e-4)
    g = g.double().cpu().numpy()
    errs = " ".join(f"{n}={np.linalg.norm(g[a:b] - gr[a:b]) / max(np.linalg.norm(gr[a:b]), 1e-30):.1e}"
                    for n, a, b in segs)
    print(f"N={N} B={B} loss_rel={abs(l - lr) / abs(lr):.1e} {errs}", flush=True)
for step, exact in [(0.01, 0), (0.01, 1), (0.005, 0)]:
    P = net.init_params(123, "cpu")
    hist, info = pkg.slbfgs_solve(net, P, X, Y, max_epochs=2, tol=0.0, lam=1e-4, M=10, L=10, b=256, b_H=128,
                                  step=step, hvp_exact=exact)
    print(f"slbfgs step={step} exact={exact}: loss {hist['loss']} pairs {hist['accepted']} evals {info.n_evals}",
          flush=True)
