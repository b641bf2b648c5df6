"""Generate the committed golden fixtures (tests/golden/*.npz) from the CPU oracle.

The oracle is itself pinned against (a) torch fp64 autograd, (b) the reference's own ring_buffer.hpp
(oracle/_ref/ring_harness, compiled from /root/reference when present), (c) the reference's known-answer
tests (tests/main.cpp) and (d) the seed-123 init draws recorded in SURVEY.md §8(c); see
tests/test_oracle.py. Inputs are stored compactly: synthetic MNIST pixels as uint8 (x = k/255).

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402


def save(name, **arrs):
    np.savez_compressed(os.path.join(HERE, name), **arrs)


def main():
    # (1) loss/grad of small MLPs, seed-123 CPU init, fp64
    X, Y = O.synth_mnist(64, 784, 10, 123)
    for dims, acts, tag in [([784, 16, 10], ["relu", "linear"], "mlp784"),
                            ([784, 16, 8, 10], ["tanh", "sigmoid", "linear"], "mlp784_deep")]:
        net = O.Net(dims, acts)
        P = net.init_cpu(123)
        l, g = net.loss_grad(P, X, Y)
        save(f"{tag}.npz", dims=np.array(dims), acts=np.array([O.ACTS[a] for a in acts]), Xu8=np.round(X * 255).astype(np.uint8),
             Y=Y.astype(np.uint8), P=P, loss=np.array(l), grad=g)
    rng = np.random.default_rng(5)
    Xs = rng.standard_normal((64, 32))
    Ys = np.zeros((64, 10))
    Ys[np.arange(64), rng.integers(0, 10, 64)] = 1
    net = O.Net([32, 16, 10], ["relu", "linear"])
    P = net.init_cpu(123)
    l, g = net.loss_grad(P, Xs, Ys)
    save("mlp32.npz", dims=np.array([32, 16, 10]), acts=np.array([2, 0]), X=Xs, Y=Ys, P=P, loss=np.array(l), grad=g)

    # (2) two-loop: n=1000, k in {0,1,5,10}; mode 0 (CPU), 1 (S-LBFGS), 2 (CUDA)
    n = 1000
    rng = np.random.default_rng(11)
    d = rng.uniform(0.5, 2.0, n)
    S = rng.standard_normal((10, n))
    Yv = S * d + 0.01 * rng.standard_normal((10, n))
    rho = 1.0 / np.einsum("ij,ij->i", S, Yv)
    gv = rng.standard_normal(n)
    out = {}
    for k in (0, 1, 5, 10):
        for mode in (0, 1, 2):
            out[f"dir_k{k}_m{mode}"] = O.two_loop(mode, S[:k] if k else np.zeros((0, n)), Yv[:k], rho[:k], gv)
    save("two_loop.npz", S=S, Y=Yv, rho=rho, g=gv, **out)

    # (3) first 20 L-BFGS iterations (Wolfe, CPU semantics) on 784-32-10, N=256, m=10
    X, Y = O.synth_mnist(256, 784, 10, 123)
    net = O.Net([784, 32, 10], ["relu", "linear"])
    P = net.init_cpu(123)
    _, rec, info = net.lbfgs_wolfe(P, X, Y, m=10, max_iters=20)
    save("lbfgs_traj.npz", rec=rec, n_fwd=np.array(info["n_fwd"]), n_bwd=np.array(info["n_bwd"]))

    # (4) S-LBFGS: sampled indices N=1000, b=32 and a 2-epoch run on 784-16-10, N=512
    idx = O.sample_indices(1000, 32, 123, calls=4)
    X, Y = O.synth_mnist(512, 784, 10, 123)
    net = O.Net([784, 16, 10], ["relu", "linear"])
    P = net.init_cpu(123)
    _, srec, sidx = net.slbfgs(P, X, Y, epochs=2, tol=0.0, M=5, L=4, b=32, bH=16, step=0.02, lam=1e-4,
                               want_idx=True)
    save("slbfgs.npz", idx=idx, rec=srec, sampled=sidx.astype(np.int32))

    # (5) ring-buffer trace (cap 3, 8 pushes) — from the reference's own header when available
    heads, contents = O.ring_trace(3, 8)
    save("ring.npz", heads=heads, contents=contents)

    # (6) init draws, both streams (first 16 of each layer segment start)
    net = O.Net([784, 128, 10], ["relu", "linear"])
    save("init.npz", cpu=net.init_cpu(123)[:256], cuda=net.init_cuda(123)[:256])
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
