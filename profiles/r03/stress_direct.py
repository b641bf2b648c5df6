"""Round-3: stress the direct-operand forward GEMM (an earlier run on one box gave NaN gradients twice, later
runs never): many evaluations on two contexts with interleaved launches (two streams), every result compared
bitwise with the LDS-DMA kernel's; S-LBFGS with the twin. Prints the number of mismatches."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

pkg = __graft_entry__.load_package()
Xh, Yh = pkg.synth_mnist(2048)
X, Y = torch.from_numpy(Xh).cuda(), torch.from_numpy(Yh).cuda()
ctx = pkg.Context(0)
ctx2 = pkg.Context(0, use_torch_stream=False)
t0 = time.time()
bad = 0
total = 0
for dims, acts in [([784, 16, 10], ["relu", "linear"]), ([784, 512, 256, 10], ["relu", "relu", "linear"]),
                   ([784, 128, 10], ["relu", "linear"])]:
    os.environ["LBF_GEMM_DIRECT"] = "0"
    ref_net = pkg.Mlp(ctx, dims, acts)
    P = ref_net.init_params(5, "cpu")
    refs = {B: ref_net.loss_grad(P, X[:B], Y[:B], l2=1e-4)[1].clone() for B in (16, 32, 96, 256, 2048)}
    os.environ["LBF_GEMM_DIRECT"] = "1"
    n1, n2 = pkg.Mlp(ctx, dims, acts), pkg.Mlp(ctx2, dims, acts)
    g1s = {B: n1.new_params() for B in refs}
    g2s = {B: n2.new_params() for B in refs}
    for rep in range(60):
        for B in refs:
            n1.loss_grad(P, X[:B], Y[:B], l2=1e-4, grad=g1s[B])
            n2.loss_grad(P, X[:B], Y[:B], l2=1e-4, grad=g2s[B])
            total += 2
            if not torch.equal(g1s[B], refs[B]):
                bad += 1
                print("mismatch ctx1", dims, B, rep, bool(torch.isfinite(g1s[B]).all()), flush=True)
            if not torch.equal(g2s[B], refs[B]):
                bad += 1
                print("mismatch ctx2", dims, B, rep, bool(torch.isfinite(g2s[B]).all()), flush=True)
    print(dims, "done", total, "evaluations", bad, "mismatches", round(time.time() - t0, 1), "s", flush=True)
kw = dict(M=5, L=4, b=32, b_H=16, step=0.02, max_epochs=2, tol=0.0, lam=1e-4)
os.environ["LBF_GEMM_DIRECT"] = os.environ.get("STRESS_SLBFGS_DIRECT", "1")
print("S-LBFGS with LBF_GEMM_DIRECT", os.environ["LBF_GEMM_DIRECT"], flush=True)
for rep in range(10):
    net = pkg.Mlp(ctx, [784, 16, 10], ["relu", "linear"])
    P = net.init_params(123, "cpu")
    hist, info = pkg.slbfgs_solve(net, P, X[:512], Y[:512], **kw)
    ok = np.array_equal(hist["accepted"], [2, 5]) and np.isfinite(hist["loss"]).all()
    bad += 0 if ok else 1
    if not ok:
        print("slbfgs mismatch", rep, hist["loss"], hist["accepted"], flush=True)
print("TOTAL mismatches", bad, flush=True)
