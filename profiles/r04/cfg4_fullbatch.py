"""Config 4 under replicated data parallelism, per-rank work measured on one GPU: the full-batch gradient
at the epoch's anchor (s_lbfgs.hpp:206, 274-284), the only evaluation the replicated route shards, at the
1-rank (60000 rows) and 8-rank (7500 rows) share of 784-512-256-10. Prints one JSON line; the projection
 is epoch(1 GPU) - t(60000) + t(7500) + the all-reduce of n + 2 floats."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

pkg = __graft_entry__.load_package()
ctx = pkg.Context(0)
dims, acts = [784, 512, 256, 10], ["relu", "relu", "linear"]
Xh, Yh = pkg.synth_mnist(60000, 784, 10, 123)
X, Y = torch.from_numpy(Xh).cuda(), torch.from_numpy(Yh).cuda()
net = pkg.Mlp(ctx, dims, acts)
P = net.init_params(123, "cpu")
out = {"bench": "cfg4_fullbatch", "dims": dims}
for rows in (60000, 30000, 15000, 7500):
    Xs, Ys = X[:rows].contiguous(), Y[:rows].contiguous()
    for _ in range(3):
        net.loss_grad(P, Xs, Ys, inv_scale=1.0 / 60000, l2=1e-4)
    torch.cuda.synchronize()
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        net.loss_grad(P, Xs, Ys, inv_scale=1.0 / 60000, l2=1e-4)
    torch.cuda.synchronize()
    out[f"loss_grad_ms_{rows}"] = round((time.perf_counter() - t0) / reps * 1e3, 4)
print(json.dumps(out), flush=True)
