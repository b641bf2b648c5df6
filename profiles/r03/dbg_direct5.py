"""Round-3 debug 5: where the intermittent NaN of the direct-operand forward shows up in loss_grad (784-16-10)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

pkg = __graft_entry__.load_package()
Xh, Yh = pkg.synth_mnist(2048)
X, Y = torch.from_numpy(Xh).cuda(), torch.from_numpy(Yh).cuda()
ctx = pkg.Context(0)
dims, acts = [784, 16, 10], ["relu", "linear"]
segs = [(0, 784 * 16), (784 * 16, 785 * 16), (785 * 16, 785 * 16 + 160), (785 * 16 + 160, 785 * 16 + 170)]
for mode in ("direct", "direct_nohead", "lds"):
    os.environ["LBF_GEMM_DIRECT"] = "0" if mode == "lds" else "1"
    os.environ["LBF_NO_HEAD"] = "1" if mode == "direct_nohead" else "0"
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(5, "cpu")
    nbad, first = 0, None
    for rep in range(300):
        B = (16, 32, 96, 256, 2048)[rep % 5]
        loss, g = net.loss_grad(P, X[:B], Y[:B], l2=1e-4)
        if not torch.isfinite(g).all():
            nbad += 1
            if first is None:
                first = (rep, B, loss, [int((~torch.isfinite(g[a:b])).sum()) for a, b in segs])
    print(mode, "bad", nbad, "of 300; first", first, flush=True)
