"""Round-3 debug, part 2: where the direct-operand forward makes the gradient NaN at B < 32 rows."""
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
for dims, acts in [([784, 16, 10], ["relu", "linear"]), ([784, 512, 256, 10], ["relu", "relu", "linear"])]:
    for B in (8, 16, 24, 31, 32, 33, 48):
        r = []
        for flag in ("0", "1"):
            os.environ["LBF_GEMM_DIRECT"] = flag
            net = pkg.Mlp(ctx, dims, acts)
            P = net.init_params(123, "cpu")
            out = net.forward(P, X[:B])
            loss, g = net.loss_grad(P, X[:B], Y[:B], l2=1e-4)
            r.append((out.clone(), loss, g.clone(), net))
        segs, off = [], 0
        for i in range(len(dims) - 1):
            n = (dims[i] + 1) * dims[i + 1]
            segs.append((off, off + n))
            off += n
        g0, g1 = r[0][2], r[1][2]
        bad = [(i, int(torch.isnan(g1[a:b]).sum()), float((g0[a:b] - g1[a:b]).abs().max())) for i, (a, b) in enumerate(segs)]
        print(dims, B, "fwd equal", bool(torch.equal(r[0][0], r[1][0])), "loss", r[0][1] == r[1][1], "grad segs (nan, maxdiff)",
              bad, flush=True)
