"""Round-3 debug, part 3: is the direct-operand NaN reproducible, and does it need two streams?"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

pkg = __graft_entry__.load_package()
dims, acts = [784, 16, 10], ["relu", "linear"]
Xh, Yh = pkg.synth_mnist(512)
X, Y = torch.from_numpy(Xh).cuda(), torch.from_numpy(Yh).cuda()
ctx = pkg.Context(0)
os.environ["LBF_GEMM_DIRECT"] = "1"
for rep in range(3):
    for B in (16, 32, 512):
        net = pkg.Mlp(ctx, dims, acts)
        P = net.init_params(123, "cpu")
        loss, g = net.loss_grad(P, X[:B], Y[:B], l2=1e-4)
        loss2, g2 = net.loss_grad(P, X[:B], Y[:B], l2=1e-4)
        print(rep, B, loss, bool(torch.isfinite(g).all()), bool(torch.isfinite(g2).all()), bool(torch.equal(g, g2)),
              flush=True)
# two contexts (two streams), launches interleaved from one thread
ctx2 = pkg.Context(0, use_torch_stream=False)
n1, n2 = pkg.Mlp(ctx, dims, acts), pkg.Mlp(ctx2, dims, acts)
P = n1.init_params(123, "cpu")
for B in (16, 32):
    l1, g1 = n1.loss_grad(P, X[:B], Y[:B], l2=1e-4)
    l2, g2 = n2.loss_grad(P, X[:B], Y[:B], l2=1e-4)
    print("two ctx", B, l1, l2, bool(torch.isfinite(g1).all()), bool(torch.isfinite(g2).all()), bool(torch.equal(g1, g2)),
          flush=True)
kw = dict(M=5, L=4, b=32, b_H=16, step=0.02, max_epochs=2, tol=0.0, lam=1e-4)
for anchor in ("0", "1"):
    os.environ["LBF_SLBFGS_ANCHOR"] = anchor
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    hist, info = pkg.slbfgs_solve(net, P, X, Y, pair_trace=4, **kw)
    print("anchor", anchor, hist["loss"], hist["accepted"], flush=True)
