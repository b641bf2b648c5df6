"""Diagnostic: per-layer gradient error of 784-128-64-10 vs the oracle across N and route knobs."""
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
dims, acts = [784, 128, 64, 10], ["relu", "relu", "linear"]
Xh, Yh = pkg.synth_mnist(60000)
X, Y = torch.from_numpy(Xh).cuda(), torch.from_numpy(Yh).cuda()
X64, Y64 = Xh.astype(np.float64), Yh.astype(np.float64)
ctx = pkg.Context(0)
onet = O.Net(dims, acts)
segs = []
off = 0
for l in range(3):
    i, o = dims[l], dims[l + 1]
    segs.append((f"W{l}", off, off + i * o))
    segs.append((f"b{l}", off + i * o, off + (i + 1) * o))
    off += (i + 1) * o
variants = [{}, {"LBF_NO_FOLD": "1"}, {"LBF_DW_TILE64": "0"}, {"LBF_NO_GEMM_HEAD": "1"}, {"LBF_NO_HEAD": "1"}]
for N in [int(a) for a in sys.argv[1:]] or [1000, 8192, 16384, 16416, 20000, 30000, 60000]:
    P = None
    ref = None
    for v in variants:
        for k in ("LBF_NO_FOLD", "LBF_DW_TILE64", "LBF_NO_GEMM_HEAD", "LBF_NO_HEAD"):
            os.environ.pop(k, None)
        os.environ.update(v)
        net = pkg.Mlp(ctx, dims, acts)
        if P is None:
            P = net.init_params(123, "cpu")
            ref = onet.loss_grad(P.double().cpu().numpy(), X64[:N], Y64[:N])
        l, g = net.loss_grad(P, X[:N], Y[:N])
        g = g.double().cpu().numpy()
        errs = " ".join(f"{name}={np.linalg.norm(g[a:b] - ref[1][a:b]) / max(np.linalg.norm(ref[1][a:b]), 1e-30):.1e}"
                        for name, a, b in segs)
        print(f"N={N} {v} loss_rel={abs(l - ref[0]) / abs(ref[0]):.1e} {errs}", flush=True)
        del net
