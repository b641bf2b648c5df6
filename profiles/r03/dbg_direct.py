"""Round-3 debug: test_dp_slbfgs_equals_single failed with the direct-operand GEMM (single route: 0 pairs
accepted). Runs the single route with LBF_GEMM_DIRECT 0/1 x LBF_SLBFGS_TWIN 0/1 and prints losses / pairs,
plus loss_grad of the b = 32 / 16 / 512 batches direct vs LDS-DMA."""
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
for B in (16, 32, 512):
    r = []
    for flag in ("0", "1"):
        os.environ["LBF_GEMM_DIRECT"] = flag
        net = pkg.Mlp(ctx, dims, acts)
        P = net.init_params(123, "cpu")
        loss, g = net.loss_grad(P, X[:B], Y[:B], l2=1e-4)
        r.append((loss, g.clone()))
    d = (r[0][1] - r[1][1]).abs().max().item()
    print(f"B={B}: loss {r[0][0]!r} vs {r[1][0]!r}, max |dg| {d:.3e}, finite {bool(torch.isfinite(r[1][1]).all())}",
          flush=True)
kw = dict(M=5, L=4, b=32, b_H=16, step=0.02, max_epochs=2, tol=0.0, lam=1e-4)
for direct in ("0", "1"):
    for twin in ("0", "1"):
        os.environ["LBF_GEMM_DIRECT"] = direct
        os.environ["LBF_SLBFGS_TWIN"] = twin
        net = pkg.Mlp(ctx, dims, acts)
        P = net.init_params(123, "cpu")
        hist, info = pkg.slbfgs_solve(net, P, X, Y, pair_trace=20, **kw)
        print(f"direct={direct} twin={twin}: loss {hist['loss']}, accepted {hist['accepted']}", flush=True)
        for row in hist["pairs"][:4]:
            print("   ", np.array2string(np.asarray(row), precision=4), flush=True)
