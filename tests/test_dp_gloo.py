"""World-size-2 data-parallel tests on CPU (gloo), covering the N>1 decomposition the GPU path uses:
contiguous sample shards, one all-reduce of [grad | loss] per evaluation scaled by 1/N_global, the
optimizer state replicated on every rank (identical inputs -> identical trajectories), the S-LBFGS
minibatch slicing, and the communicator-id broadcast. The per-rank evaluations use the oracle (the
CPU restatement); the GPU ranks run the same decomposition with RCCL (lbfgs-ffnn_amd/csrc/runtime.cpp).
"""
import os
import sys
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _setup(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.lib()
    return O


def dp_loss_grad(O, net, P, X, Y, N_global, rank, world):
    """Local shard -> sum over ranks: grad = sum_r (N_r / N) * mean-grad_r (== RCCL all-reduce of the
    shard sums already scaled by 1/N_global), loss likewise; split fp64 loss as hi/lo fp32 words
    exactly like pack_hilo() before the all-reduce."""
    lo, hi = N_global * rank // world, N_global * (rank + 1) // world
    l, g = net.loss_grad(P, X[lo:hi], Y[lo:hi])
    w = (hi - lo) / N_global
    buf = torch.from_numpy(np.concatenate([g * w, [l * w]]))
    dist.all_reduce(buf)
    out = buf.numpy()
    return float(out[-1]), out[:-1].copy()


def wolfe_lbfgs(O, f_g, x, m, iters, c1=1e-4, c2=0.9, rho=0.5, max_ls=50):
    """Python restatement of the cached-evaluation Wolfe L-BFGS the HIP driver runs
    (lbfgs.hpp:38-100 + full_batch_minimizer.hpp:126-157)."""
    S, Yh, R = [], [], []
    loss, g = f_g(x)
    losses = []
    for it in range(iters):
        k = len(S)
        p = O.two_loop(0, np.array(S) if k else np.zeros((0, len(x))), np.array(Yh) if k else None,
                       np.array(R), g) if k else -g
        if it == 0:
            a = min(1.0, 1.0 / np.linalg.norm(g))
            ln, gn = f_g(x + a * p)
        else:
            gfo = g @ p
            a, amin, amax = 1.0, 0.0, np.inf
            for _ in range(max_ls):
                ln, gn = f_g(x + a * p)
                if ln > loss + c1 * a * gfo:
                    amax = a
                    a = rho * (amin + amax)
                    continue
                if gn @ p < c2 * gfo:
                    amin = a
                    a = 2 * a if amax == np.inf else rho * (amin + amax)
                    continue
                break
        xn = x + a * p
        s, y = xn - x, gn - g
        if y @ s > 1e-10:
            S.append(s)
            Yh.append(y)
            R.append(1.0 / (y @ s))
            if len(S) > m:
                S.pop(0), Yh.pop(0), R.pop(0)
        x, g, loss = xn, gn, ln
        losses.append(loss)
    return x, np.array(losses)


def _worker(rank, world, port, outdir):
    O = _setup(rank, world, port)
    X, Y = O.synth_mnist(400, 784, 10, 123)
    net = O.Net([784, 24, 10], ["relu", "linear"])
    P = net.init_cpu(123)
    # (1) sharded evaluation == full batch
    l, g = dp_loss_grad(O, net, P, X, Y, 400, rank, world)
    # (2) replicated optimizer on the DP objective
    x, losses = wolfe_lbfgs(O, lambda w: dp_loss_grad(O, net, w, X, Y, 400, rank, world), P.copy(), 10, 8)
    # (3) communicator id broadcast (the RCCL unique id travels the same way)
    uid = [os.urandom(128) if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    # (4) S-LBFGS minibatch slicing across ranks (solvers.cpp: [b*r/p, b*(r+1)/p))
    idx = O.sample_indices(400, 37, 123, 1)[0]
    mine = idx[37 * rank // world: 37 * (rank + 1) // world]
    np.savez(os.path.join(outdir, f"r{rank}.npz"), l=l, g=g, x=x, losses=losses, uid=np.frombuffer(uid[0], np.uint8),
             mine=mine)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_data_parallel_gloo(world, O):
    port = 29500 + (os.getpid() % 1000)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, port, d), nprocs=world, join=True)
        r = [np.load(os.path.join(d, f"r{i}.npz")) for i in range(world)]
    X, Y = O.synth_mnist(400, 784, 10, 123)
    net = O.Net([784, 24, 10], ["relu", "linear"])
    P = net.init_cpu(123)
    l_full, g_full = net.loss_grad(P, X, Y)
    for ri in r:
        assert abs(float(ri["l"]) - l_full) <= 1e-12 * abs(l_full)
        assert np.allclose(ri["g"], g_full, rtol=1e-10, atol=1e-14)
    # identical state on every rank
    assert np.array_equal(r[0]["x"], r[1]["x"])
    assert np.array_equal(r[0]["uid"], r[1]["uid"])
    # DP trajectory == single-process reference trajectory (oracle lbfgs_wolfe)
    _, rec, _ = net.lbfgs_wolfe(P, X, Y, m=10, max_iters=8)
    assert np.allclose(r[0]["losses"], rec[:, 0], rtol=1e-8)
    # minibatch slices partition the sampled list
    idx = O.sample_indices(400, 37, 123, 1)[0]
    assert np.array_equal(np.concatenate([ri["mine"] for ri in r]), idx)
