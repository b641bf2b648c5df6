"""Print the engine's split-K plan (LBF_SHOW_PLAN=1, stderr) for cfg 5 (4096-2048-1024-1) at several batch sizes:
which N engages the N = 1,000,000 route's tiles and split counts (tests/test_gpu_configs.py). Run on a GPU box:
LBF_SHOW_PLAN=1 python profiles/r06/show_plan_cfg5.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
ctx = pkg.Context(0)
net = pkg.Mlp(ctx, [4096, 2048, 1024, 1], ["relu", "relu", "linear"])
P = net.init_params(123, "cpu")
for N in (128, 2048, 4096, 8192, 16384, 20000, 24576, 28672, 32768, 36864, 40000, 1_000_000):
    X = torch.zeros((N, 4096), device="cuda")
    Y = torch.zeros((N, 1), device="cuda")
    net.loss_grad(P, X, Y)
    torch.cuda.synchronize()
    del X, Y
    print(f"N = {N} planned", flush=True)
