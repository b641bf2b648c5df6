"""The data-parallel evaluation path on ONE GPU, through a 1-rank RCCL communicator.

`lbf_comm_init(ctx, 1, 0, id)` creates a real RCCL communicator, and every evaluation then takes the
multi-rank route of runtime.cpp (per-rank reduce -> fp32 (hi, lo) loss words -> ncclAllReduce over
[grad | hi | lo] -> tail / finalize over the reduced buffer) — the code the driver's 2/4/8-GPU bench
runs, minus the cross-GPU hop. A 1-rank all-reduce is the identity, so the results must equal the
single-GPU path: gradients bit for bit, losses to the (hi, lo) split's 2^-48, and whole L-BFGS /
S-LBFGS trajectories with identical line-search decisions.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()


def host(t):
    return t.double().cpu().numpy()


@pytest.fixture(scope="module")
def dp_ctx(pkg):
    c = pkg.Context(0)
    c.comm_init(1, 0, pkg.Context.unique_id())
    return c


def test_allreduce_one_rank_is_identity(dp_ctx):
    t = torch.arange(1000, dtype=torch.float32, device="cuda") * 0.37
    ref = t.clone()
    dp_ctx.allreduce_(t)
    torch.cuda.synchronize()
    assert torch.equal(t, ref)


@pytest.mark.parametrize("dims,acts", [([784, 128, 10], ["relu", "linear"]),
                                       ([784, 128, 64, 10], ["relu", "relu", "linear"]),
                                       ([784, 300, 20], ["relu", "linear"])])
@pytest.mark.parametrize("N", [257, 7500])
def test_dp_loss_grad_equals_single(ctx, dp_ctx, pkg, dims, acts, N):
    Xh, Yh = pkg.synth_mnist(N, dims[0], dims[-1])
    X, Y = dev(Xh), dev(Yh)
    net1 = pkg.Mlp(ctx, dims, acts)
    netd = pkg.Mlp(dp_ctx, dims, acts)
    P = net1.init_params(123, "cpu")
    l1, g1 = net1.loss_grad(P, X, Y, inv_scale=1.0 / N)
    ld, gd = netd.loss_grad(P, X, Y, inv_scale=1.0 / N)
    assert torch.equal(g1, gd)
    assert abs(l1 - ld) <= 1e-12 * abs(l1)


@pytest.mark.parametrize("line_search", ["wolfe", "armijo"])
def test_dp_lbfgs_trajectory_equals_single(ctx, dp_ctx, pkg, line_search):
    """Speculative L-BFGS with the fused tail over the all-reduced buffer (runtime.cpp DP branch)."""
    dims, acts = [784, 64, 10], ["relu", "linear"]
    Xh, Yh = pkg.synth_mnist(2048)
    out = []
    for c in (ctx, dp_ctx):
        net = pkg.Mlp(c, dims, acts)
        P = net.init_params(7, "cpu")
        hist, info = pkg.lbfgs_solve(net, P, dev(Xh), dev(Yh), line_search=line_search, m=10, max_iters=30,
                                     tol=0.0)
        out.append((hist, info, host(P)))
    (h1, i1, P1), (hd, idd, Pd) = out
    assert np.array_equal(h1["ls_trials"], hd["ls_trials"])
    assert np.array_equal(h1["accepted"], hd["accepted"])
    r = np.abs(h1["loss"] - hd["loss"]) / np.abs(h1["loss"])
    assert r.max() <= 1e-9, r
    assert np.linalg.norm(P1 - Pd) <= 1e-6 * np.linalg.norm(P1)


def test_dp_lbfgs_full_size(ctx, dp_ctx, pkg):
    """cfg-2 shape at an 8-rank shard size (7500 rows), 10 iterations: DP route == single route."""
    dims, acts = [784, 128, 10], ["relu", "linear"]
    Xh, Yh = pkg.synth_mnist(60000)
    X, Y = dev(Xh[:7500]), dev(Yh[:7500])
    out = []
    for c in (ctx, dp_ctx):
        net = pkg.Mlp(c, dims, acts)
        P = net.init_params(123, "cpu")
        hist, info = pkg.lbfgs_solve(net, P, X, Y, n_global=7500, m=10, max_iters=10, tol=0.0)
        out.append(hist)
    assert np.array_equal(out[0]["ls_trials"], out[1]["ls_trials"])
    assert np.allclose(out[0]["loss"], out[1]["loss"], rtol=1e-9, atol=0)


@pytest.mark.parametrize("dp_mode", ["sliced", "replicated"])
def test_dp_slbfgs_equals_single(ctx, dp_ctx, pkg, dp_mode):
    """Both S-LBFGS data-parallel modes through a 1-rank communicator against the single route: sliced (every
    inner step's gradients through the collective) and replicated (the inner steps without it, only the
    epoch's full-batch gradient through it)."""
    dims, acts = [784, 16, 10], ["relu", "linear"]
    Xh, Yh = pkg.synth_mnist(512)
    kw = dict(M=5, L=4, b=32, b_H=16, step=0.02, max_epochs=2, tol=0.0, lam=1e-4, dp_mode=dp_mode)
    out = []
    for c in (ctx, dp_ctx):
        net = pkg.Mlp(c, dims, acts)
        P = net.init_params(123, "cpu")
        hist, info = pkg.slbfgs_solve(net, P, dev(Xh), dev(Yh), **kw)
        out.append((hist, host(P)))
    (h1, P1), (hd, Pd) = out
    assert np.array_equal(h1["accepted"], hd["accepted"])
    assert np.allclose(h1["loss"], hd["loss"], rtol=1e-9, atol=0)
    assert np.linalg.norm(P1 - Pd) <= 1e-6 * np.linalg.norm(P1)


@pytest.mark.parametrize("dp_mode", ["sliced", "replicated"])
def test_dp_slbfgs_cfg4_bitwise(ctx, dp_ctx, pkg, dp_mode):
    """BASELINE cfg 4's shape (784-512-256-10, b = 256, b_H = 128, L = M = 10) for two epochs over 12800 rows:
    the data-parallel routes against the single route, the same parameters bit for bit (s_lbfgs.hpp:218-262).
    Sliced: both minibatch gradients of a step in one [g(w_t) | g(w)] all-reduce, the twin's anchor gradients
    one step ahead, the FD pair in one [g(u+eps s) | g(u-eps s)] all-reduce. Replicated: the whole inner-step
    chain without a collective (the free-running twin included), the full-batch gradient at each anchor
    through the collective."""
    dims, acts = [784, 512, 256, 10], ["relu", "relu", "linear"]
    Xh, Yh = pkg.synth_mnist(12800)
    X, Y = dev(Xh), dev(Yh)
    kw = dict(M=10, L=10, b=256, b_H=128, step=0.005, max_epochs=2, tol=0.0, lam=1e-4, dp_mode=dp_mode)
    out = []
    for c in (ctx, dp_ctx):
        net = pkg.Mlp(c, dims, acts)
        P = net.init_params(123, "cpu")
        hist, info = pkg.slbfgs_solve(net, P, X, Y, **kw)
        out.append((hist, P, info))
    (h1, P1, i1), (hd, Pd, idd) = out
    assert torch.equal(P1, Pd)
    assert np.array_equal(h1["accepted"], hd["accepted"])
    assert i1.n_evals == idd.n_evals and i1.n_rows == idd.n_rows
    assert np.all(np.abs(h1["loss"] - hd["loss"]) <= 1e-12 * np.abs(h1["loss"]))


def test_batch_grads_equal_per_minibatch_loss_grad(ctx, pkg):
    """lbf_mlp_batch_grads (the S-LBFGS epoch's anchor gradients in one evaluation) against lbf_mlp_loss_grad on
    each minibatch: the same sums in another order (one K split per minibatch, the unfused output layer),
    so equal to fp32 rounding: max |diff| <= 1e-5 max |g| per minibatch."""
    dims, acts = [784, 512, 256, 10], ["relu", "relu", "linear"]
    nmb, cnt = 6, 256
    Xh, Yh = pkg.synth_mnist(nmb * cnt)
    X, Y = dev(Xh), dev(Yh)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(7, "cpu")
    G = net.batch_grads(P, X, Y, nmb, inv_scale=1.0 / cnt, l2=1e-4)
    for t in range(nmb):
        _, g = net.loss_grad(P, X[t * cnt:(t + 1) * cnt], Y[t * cnt:(t + 1) * cnt], inv_scale=1.0 / cnt, l2=1e-4)
        ref = host(g)
        err = np.abs(host(G[t]) - ref).max()
        assert err <= 1e-5 * np.abs(ref).max(), (t, err, np.abs(ref).max())


@pytest.mark.parametrize("dims,acts,B", [([784, 128, 10], ["relu", "linear"], 7500),   # 32x128 EPI_HEAD + fold
                                         ([784, 128, 10], ["relu", "linear"], 1000),
                                         ([784, 512, 256, 10], ["relu", "tanh", "linear"], 256),  # split-K
                                         ([784, 512, 256, 10], ["relu", "relu", "linear"], 96),
                                         # the next split GEMM forms its A from the previous layer's slabs
                                         # (activation inside the prologue; 13 slabs = two rounds at B = 96)
                                         ([784, 512, 256, 10], ["tanh", "relu", "linear"], 256),
                                         ([784, 512, 256, 128, 10], ["relu", "sigmoid", "relu", "linear"], 256),
                                         ([784, 128, 64, 10], ["sigmoid", "relu", "linear"], 333),
                                         # N = 16 < the tile width, EPI_HEAD with the 16-column fold, M < 32: the
                                         # epilogue consumes the whole tile's accumulators (rows >= M, columns
                                         # >= N must be exact zeros; they were copies of the clamped edge once,
                                         # and the fold's rows came out NaN)
                                         ([784, 16, 10], ["relu", "linear"], 16),
                                         ([784, 16, 10], ["relu", "linear"], 2048)])
def test_small_tile_shapes_match_oracle(ctx, pkg, O, dims, acts, B):
    """The 32 x 128 forward tile's edge shapes (EPI_HEAD with the fold, plain forward, split-K slabs, ragged
    rows, N = 16 below the tile width with M < 32: the epilogue consumes the whole tile's accumulators, so rows
    >= M and columns >= N must be exact zeros) against the fp64 oracle, finite, and bitwise reproducible."""
    Xh, Yh = pkg.synth_mnist(B)
    X, Y = dev(Xh), dev(Yh)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(21, "cpu")
    loss, g = net.loss_grad(P, X, Y, l2=1e-4)
    g = g.clone()
    loss2, g2 = net.loss_grad(P, X, Y, l2=1e-4)
    assert loss == loss2 and torch.equal(g, g2)
    assert bool(torch.isfinite(g).all())
    onet = O.Net(dims, acts)
    P64 = host(P)
    l_ref, g_ref = onet.loss_grad(P64, Xh.astype(np.float64), Yh.astype(np.float64), lam=1e-4)
    assert abs(loss - l_ref) <= 1e-5 * abs(l_ref)
    assert np.linalg.norm(host(g) - g_ref) <= 1e-4 * np.linalg.norm(g_ref)
