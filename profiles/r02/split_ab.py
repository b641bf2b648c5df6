"""A/B of the GEMM arithmetic (LBF_GEMM_SPLIT = 0 exact fp32 MFMA, 6 / 9 = split-bf16 products):
loss/gradient error vs the fp64 oracle at cfg 2/3 full size, next to the exact-fp32 route's own error."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

if len(sys.argv) > 1 and sys.argv[1] == "child":
    import torch
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    O = __graft_entry__.load_oracle()
    N = int(sys.argv[2])
    dims = [int(x) for x in sys.argv[3].split(",")]
    acts = sys.argv[4].split(",")
    Xh, Yh = pkg.synth_mnist(N, dims[0], dims[-1])
    ctx = pkg.Context(0)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    l, g = net.loss_grad(P, torch.from_numpy(Xh).cuda(), torch.from_numpy(Yh).cuda())
    lr, gr = O.Net(dims, acts).loss_grad(P.double().cpu().numpy(), Xh.astype(np.float64), Yh.astype(np.float64))
    g = g.double().cpu().numpy()
    print(json.dumps(dict(loss_rel=abs(l - lr) / abs(lr), grad_rel=float(np.linalg.norm(g - gr) / np.linalg.norm(gr)))))
    sys.exit(0)

for dims, acts in [("784,128,10", "relu,linear"), ("784,128,64,10", "relu,relu,linear")]:
    for mode in ("0", "6", "9"):
        env = dict(os.environ, LBF_GEMM_SPLIT=mode)
        out = subprocess.run([sys.executable, __file__, "child", "60000", dims, acts], env=env, capture_output=True,
                             text=True, timeout=300)
        print(dims, "split", mode, out.stdout.strip().splitlines()[-1] if out.stdout.strip() else out.stderr[-2000:],
              flush=True)
