"""Round-3 diagnostic, part 2 (after diag_nan.py): the FIRST curvature-pair candidate of the cfg-4 S-LBFGS epoch
(step 0.01, epoch 0, t = 20) already differs between the device (y.s = 0.040, |y| = 0.93, equal to the exact
R-operator HVP) and the fp64 oracle (y.s = 0.205, |y| = 18.9). Here the SAME (u, s, Hessian rows), taken
from the fp64 oracle's run, go through every HVP implementation:
  oracle fp64 FD, oracle fp32 FD, device FD (lbf_mlp_fd_hvp), device exact HVP (lbf_mlp_hvp),
and the ReLU units whose pre-activation changes sign between u - eps s and u + eps s are counted (fp64 numpy):
finite_difference_hvp_batch (s_lbfgs.hpp:88-101) differences the gradient across those kinks, where the
gradient jumps, so each crossing adds a term of order |jump| / (2 eps) that the Hessian does not have.
"""
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
N, b, bH, L, STEP, EPS, LAM = 60000, 256, 128, 10, 0.01, 1e-4, 1e-4
Xh, Yh = pkg.synth_mnist(N)
X64, Y64 = Xh.astype(np.float64), Yh.astype(np.float64)
ctx = pkg.Context(0)
net = pkg.Mlp(ctx, dims, acts)
P0 = net.init_params(123, "cpu").double().cpu().numpy()
onet = O.Net(dims, acts)
n = onet.nparams
us = np.zeros(2 * n)
_, _, idx = onet.slbfgs(P0, X64, Y64, epochs=1, tol=0.0, M=10, L=L, b=b, bH=bH, step=STEP, lam=LAM, want_idx=True,
                        pair0=us)
u, s = us[:n], us[n:]
# sampled lists in order: minibatches of steps 0..20 (b rows each), then the Hessian batch of step 20
rows = idx[21 * b: 21 * b + bH]
print(f"pair 0: |u| {np.linalg.norm(u):.4f} |s| {np.linalg.norm(s):.4e}, Hessian rows {rows[:6]}...", flush=True)

res = {}
res["oracle_fp64_fd"] = onet.fd_hvp(u, s, X64, Y64, idx=rows, lam=LAM, eps=EPS)
res["oracle_fp32_fd"] = onet.fd_hvp_f32(u, s, X64, Y64, rows, lam=LAM, eps=EPS)
X, Y = torch.from_numpy(Xh).cuda(), torch.from_numpy(Yh).cuda()
ud = torch.from_numpy(u.astype(np.float32)).cuda()
sd = torch.from_numpy(s.astype(np.float32)).cuda()
ri = torch.from_numpy(rows.astype(np.int32)).cuda()
res["device_fd"] = net.fd_hvp(ud, sd, X, Y, idx=ri, inv_scale=1.0 / bH, l2=LAM, eps=EPS).double().cpu().numpy()
res["device_exact"] = net.hvp(ud, sd, X, Y, idx=ri, inv_scale=1.0 / bH, l2=LAM).double().cpu().numpy()
for k, y in res.items():
    print(f"{k:16s} y.s {y @ s: .4e}  |y| {np.linalg.norm(y):.4e}  rel to exact "
          f"{np.linalg.norm(y - res['device_exact']) / np.linalg.norm(res['device_exact']):.3e}", flush=True)


# ReLU sign changes between u - eps s and u + eps s on the Hessian rows (fp64)
def preacts(P, x):
    out, off, a = [], 0, x
    for l in range(3):
        i, o = dims[l], dims[l + 1]
        W = P[off: off + i * o].reshape(i, o)
        bb = P[off + i * o: off + (i + 1) * o]
        z = a @ W + bb
        out.append(z)
        a = np.maximum(z, 0.0) if acts[l] == "relu" else z
        off += (i + 1) * o
    return out


xb = X64[rows]
zp, zm = preacts(u + EPS * s, xb), preacts(u - EPS * s, xb)
for l in range(2):
    flips = int(np.sum(np.sign(zp[l]) != np.sign(zm[l])))
    dz = np.abs(zp[l] - zm[l])
    print(f"layer {l}: {flips} ReLU sign flips over {zp[l].size} pre-activations; |dz| median {np.median(dz):.2e} "
          f"max {dz.max():.2e}; min |z| at u {np.abs(preacts(u, xb)[l]).min():.2e}")
# the same, for the fp32 perturbation the device and the fp32 oracle form
u32, s32 = u.astype(np.float32), s.astype(np.float32)
wp32 = (u32.astype(np.float64) + EPS * s32.astype(np.float64)).astype(np.float32).astype(np.float64)
wm32 = (u32.astype(np.float64) - EPS * s32.astype(np.float64)).astype(np.float32).astype(np.float64)
zp, zm = preacts(wp32, xb), preacts(wm32, xb)
for l in range(2):
    flips = int(np.sum(np.sign(zp[l]) != np.sign(zm[l])))
    print(f"fp32-rounded u +- eps s, layer {l}: {flips} sign flips; perturbed coordinates "
          f"{int(np.sum(wp32 != wm32))} of {n} (fp64: {int(np.sum(s != 0))})")
