"""Round-3: S-LBFGS (784-16-10, b = 32, twin stream) intermittently NaN with the direct-operand forward GEMM.
Which combination fails: {direct, LDS-DMA} x {twin, no twin, anchor precompute}, 12 runs each."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

pkg = __graft_entry__.load_package()
Xh, Yh = pkg.synth_mnist(512)
X, Y = torch.from_numpy(Xh).cuda(), torch.from_numpy(Yh).cuda()
ctx = pkg.Context(0)
kw = dict(M=5, L=4, b=32, b_H=16, step=0.02, max_epochs=2, tol=0.0, lam=1e-4)
for direct in ("1", "0"):
    for mode in ("twin", "notwin", "anchor"):
        os.environ["LBF_GEMM_DIRECT"] = direct
        os.environ["LBF_SLBFGS_TWIN"] = "0" if mode == "notwin" else "1"
        os.environ["LBF_SLBFGS_ANCHOR"] = "1" if mode == "anchor" else "0"
        bad = 0
        for rep in range(12):
            net = pkg.Mlp(ctx, [784, 16, 10], ["relu", "linear"])
            P = net.init_params(123, "cpu")
            hist, info = pkg.slbfgs_solve(net, P, X, Y, **kw)
            if not np.isfinite(hist["loss"]).all():
                bad += 1
        print(f"direct={direct} {mode}: {bad} of 12 runs NaN", flush=True)
