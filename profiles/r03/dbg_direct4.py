"""Round-3 debug 4: slab entries left unwritten by the direct kernel? (LBF_DBG_POISON_FSLAB=1 fills the forward
split-K slabs with NaN before each GEMM.)"""
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
for direct in ("0", "1"):
    os.environ["LBF_GEMM_DIRECT"] = direct
    for dims, acts in [([784, 16, 10], ["relu", "linear"]), ([784, 64, 10], ["relu", "linear"]),
                       ([784, 512, 256, 10], ["relu", "relu", "linear"])]:
        net = pkg.Mlp(ctx, dims, acts)
        P = net.init_params(5, "cpu")
        res = []
        for B in (16, 32, 96, 256, 2048):
            out = net.forward(P, X[:B])
            res.append((B, bool(torch.isfinite(out).all()), int((~torch.isfinite(out)).sum())))
        print("direct", direct, dims, res, flush=True)
