"""Round-3 diagnostic (VERDICT r02 item 6 / ADVICE medium): why does the device S-LBFGS at step 0.01 on the
cfg-4 shape (784-512-256-10, N = 60000, b = 256, b_H = 128, L = M = 10) reach NaN while the oracle's fp32
instantiation survives?

Side by side, per curvature-pair candidate (s_lbfgs.hpp:245-256): y.s, s.s, y.y, accepted, live pairs, for
  - the device (FD HVP, the reference's finite difference), the device with the exact R-operator HVP,
  - the oracle in fp64 (the reference's arithmetic) and fp32 (oracle/oracle.hpp's fp32 instantiation,
    whose GEMM sums accumulate in fp64),
plus the per-epoch loss. Same host RNG stream everywhere, so candidate i is the same (epoch, t) in every
run until the trajectories part.
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

pkg = __graft_entry__.load_package()
O = __graft_entry__.load_oracle()
dims, acts = [784, 512, 256, 10], ["relu", "relu", "linear"]
N = 60000
EPOCHS = int(os.environ.get("DIAG_EPOCHS", "2"))
STEP = float(os.environ.get("DIAG_STEP", "0.01"))
Xh, Yh = pkg.synth_mnist(N)
X, Y = torch.from_numpy(Xh).cuda(), torch.from_numpy(Yh).cuda()
ctx = pkg.Context(0)
net = pkg.Mlp(ctx, dims, acts)
kw = dict(M=10, L=10, b=256, b_H=128, step=STEP, lam=1e-4, tol=0.0, max_epochs=EPOCHS)
out = {}
for name, exact in [("device_fd", 0), ("device_exact", 1)]:
    P = net.init_params(123, "cpu")
    hist, info = pkg.slbfgs_solve(net, P, X, Y, hvp_exact=exact, pair_trace=200, **kw)
    out[name] = dict(loss=hist["loss"].tolist(), pairs=hist["pairs"].tolist())
    print(name, "epoch losses", hist["loss"], flush=True)
P0 = net.init_params(123, "cpu").double().cpu().numpy()
onet = O.Net(dims, acts)
X64, Y64 = Xh.astype(np.float64), Yh.astype(np.float64)
for name, fp32 in [("oracle_fp64", False), ("oracle_fp32", True)]:
    _, rec, _, pairs = onet.slbfgs(P0, X64, Y64, epochs=EPOCHS, tol=0.0, M=10, L=10, b=256, bH=128, step=STEP,
                                   lam=1e-4, fp32=fp32, pair_trace=200)
    out[name] = dict(loss=rec[:, 0].tolist(), pairs=pairs.tolist())
    print(name, "epoch losses", rec[:, 0], flush=True)
names = list(out)
npair = max(len(out[n]["pairs"]) for n in names)
print(f"\n{'#':>3} {'ep':>2} {'t':>4} | " + " | ".join(f"{n:^34}" for n in names))
print(f"{'':>3} {'':>2} {'':>4} | " + " | ".join(f"{'y.s':>11} {'|s|':>9} {'|y|':>9} {'k':>2}" for _ in names))
for i in range(npair):
    cells, ep, t = [], None, None
    for n in names:
        p = out[n]["pairs"]
        if i < len(p):
            r = p[i]
            ep, t = int(r[0]), int(r[1])
            cells.append(f"{r[2]:11.3e} {np.sqrt(max(r[3], 0)):9.2e} {np.sqrt(max(r[4], 0)):9.2e} {int(r[6]):2d}")
        else:
            cells.append(" " * 34)
    print(f"{i:3d} {ep:2d} {t:4d} | " + " | ".join(cells))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", f"diag_nan_step{STEP}.json"), "w"))
