"""GEMM probe (GPU box): our fwd / dW GEMMs at the cfg-2 shape and at 4x the rows (no tail effect),
beside torch's fp32 matmul (hipBLASLt / rocBLAS) on the same shapes.  python3 profiles/gemm_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402


def ev_time(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


def main():
    pkg = __graft_entry__.load_package()
    ctx = pkg.Context(0)
    dims = [int(x) for x in os.environ.get("DIMS", "784,128,10").split(",")]
    for N in [int(x) for x in os.environ.get("NS", "60000,240000").split(",")]:
        X = torch.randn(N, dims[0], device="cuda")
        Y = torch.randn(N, dims[-1], device="cuda")
        net = pkg.Mlp(ctx, dims, ["relu"] * (len(dims) - 2) + ["linear"])
        P = net.init_params(1, "cpu")
        g = net.new_params()
        net.loss_grad(P, X, Y, grad=g)
        ctx.prof_enable(True)
        for _ in range(20):
            net.loss_grad(P, X, Y, grad=g)
        prof = ctx.prof_read()
        ctx.prof_enable(False)
        for k, (ms, c) in sorted(prof.items()):
            us = ms / c * 1e3
            line = f"N={N} {k:18s} {us:9.2f} us"
            if k.startswith("gemm_"):
                l = int(k.split("[")[1][:-1])
                fl = 2.0 * N * dims[l] * dims[l + 1]
                line += f"  {fl / us / 1e6:7.1f} TF"
            print(line, flush=True)
        W = torch.randn(dims[0], dims[1], device="cuda")
        D = torch.randn(N, dims[1], device="cuda")
        fl = 2.0 * N * dims[0] * dims[1]
        t1 = ev_time(lambda: X @ W)
        t2 = ev_time(lambda: X.t() @ D)
        print(f"N={N} torch X@W      {t1:9.2f} us  {fl / t1 / 1e6:7.1f} TF", flush=True)
        print(f"N={N} torch X^T@D    {t2:9.2f} us  {fl / t2 / 1e6:7.1f} TF", flush=True)
    M = 4096
    A = torch.randn(M, M, device="cuda")
    t = ev_time(lambda: A @ A, 10)
    print(f"torch 4096^3 {t:9.2f} us {2 * M ** 3 / t / 1e6:7.1f} TF")


if __name__ == "__main__":
    main()
