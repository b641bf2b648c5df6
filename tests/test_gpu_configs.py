"""GPU parity at the shapes of BASELINE configs 3-5 (configs 1-2 are covered by test_gpu_parity.py).

cfg 3: 784-128-64-10 (ReLU, ReLU, Linear), L-BFGS m = 20.
cfg 4: S-LBFGS 784-512-256-10 (b = 256, b_H = 128, L = M = 10, step 0.02, lambda 1e-4), also through the
       data-parallel route (1-rank RCCL communicator, the code the 8-GPU config runs).
cfg 5: 4096-2048-1024-1 (ReLU, ReLU, Linear) regression on the device-generated data (synth.hip,
       restated in oracle/oracle.py), L-BFGS m = 50; oracle parity at small N, and at the full
       N = 1,000,000 the size-independent properties (directional derivative, shard sums, monotone
       Wolfe descent).
Tolerances as in test_gpu_parity.py: loss 1e-5, gradient max(1e-4, 3x the fp32
oracle's own error), trajectories 1e-3 on the early iterations with identical line-search decisions.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CFG5 = ([4096, 2048, 1024, 1], ["relu", "relu", "linear"])


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()


def host(t):
    return t.double().cpu().numpy()


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def test_cfg3_lbfgs_m20_trajectory(ctx, pkg, O):
    dims, acts = [784, 128, 64, 10], ["relu", "relu", "linear"]
    Xh, Yh = pkg.synth_mnist(512)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    P0 = host(P)
    hist, _ = pkg.lbfgs_solve(net, P, dev(Xh), dev(Yh), m=20, max_iters=25, tol=0.0)
    _, rec, _ = O.Net(dims, acts).lbfgs_wolfe(P0, Xh.astype(np.float64), Yh.astype(np.float64), m=20, max_iters=25)
    r = np.abs(hist["loss"][:10] - rec[:10, 0]) / np.abs(rec[:10, 0])
    assert r.max() <= 1e-3, r
    assert np.array_equal(hist["ls_trials"][:10], rec[:10, 4].astype(int))


@pytest.mark.parametrize("dp", [False, True])
def test_cfg4_slbfgs_shape(ctx, pkg, O, dp):
    """S-LBFGS at the cfg-4 network and hyper-parameters on 2048 samples (8 inner steps per epoch, one
    curvature pair per epoch from the second on), 2 epochs, vs the fp64 oracle."""
    dims, acts = [784, 512, 256, 10], ["relu", "relu", "linear"]
    N = 2048
    Xh, Yh = pkg.synth_mnist(N)
    c = ctx
    if dp:
        c = pkg.Context(0)
        c.comm_init(1, 0, pkg.Context.unique_id())
    net = pkg.Mlp(c, dims, acts)
    P = net.init_params(123, "cpu")
    P0 = host(P)
    kw = dict(M=10, L=10, b=256, b_H=128, step=0.02)
    hist, _ = pkg.slbfgs_solve(net, P, dev(Xh), dev(Yh), max_epochs=3, tol=0.0, lam=1e-4, **kw)
    _, rec, _ = O.Net(dims, acts).slbfgs(P0, Xh.astype(np.float64), Yh.astype(np.float64), epochs=3, tol=0.0,
                                         M=10, L=10, b=256, bH=128, step=0.02, lam=1e-4)
    r = np.abs(hist["loss"] - rec[:, 0]) / np.abs(rec[:, 0])
    assert r.max() <= 1e-3, r
    assert np.array_equal(hist["accepted"], rec[:, 3].astype(int))


def test_cfg5_synth_matches_oracle(ctx, pkg, O):
    N, In = 96, 4096
    X, Y = pkg.synth_regression(ctx, N, In)
    Xo, Yo = O.synth_regression(N, In)
    Xg, Yg = X.cpu().numpy(), Y.cpu().numpy()
    # fp64 log/sin/cos on the device vs numpy, rounded once to fp32: equal but for rare last-ulp ties
    assert np.mean(Xg == Xo) > 0.999
    assert np.max(np.abs(Xg - Xo)) <= 1e-6 * max(1.0, np.abs(Xo).max())
    assert np.max(np.abs(Yg - Yo)) <= 1e-5
    X2, Y2 = pkg.synth_regression(ctx, N, In)
    assert torch.equal(X, X2) and torch.equal(Y, Y2)


def test_cfg5_loss_grad_matches_oracle(ctx, pkg, O):
    dims, acts = CFG5
    N = 64
    X, Y = pkg.synth_regression(ctx, N, dims[0])
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    loss, g = net.loss_grad(P, X, Y)
    onet = O.Net(dims, acts)
    Xh, Yh = host(X), host(Y)
    l_ref, g_ref = onet.loss_grad(host(P), Xh, Yh)
    assert abs(loss - l_ref) <= 1e-5 * abs(l_ref)
    _, g32 = onet.loss_grad_f32(host(P), Xh, Yh)
    assert rel(host(g), g_ref) <= max(1e-4, 3.0 * rel(g32, g_ref))


def test_cfg5_loss_grad_split_plan_matches_oracle(ctx, pkg, O):
    """cfg 5 against the fp64 oracle where the N = 1,000,000 route engages: from ~8k rows the
    two wide dW GEMMs run the 1M plan's 128 x 128 tiles with the same split counts (layer 0: 33 x 16 = 528 tiles
    in 29 splits, layer 1: 17 x 8 in 15; LBF_SHOW_PLAN output in profiles/r06/), the forward GEMMs run unsplit
    128-row tiles, and the last layer's 1024 x 1 dW is split many ways; below 2048 rows (the N <= 128 tests above)
    every dW GEMM takes the small-batch 64 x 64 plan instead. Loss 1e-5, gradient 1e-4 (the full-size bounds)."""
    dims, acts = CFG5
    N = 8192
    X, Y = pkg.synth_regression(ctx, N, dims[0])
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    loss, g = net.loss_grad(P, X, Y)
    onet = O.Net(dims, acts)
    l_ref, g_ref = onet.loss_grad(host(P), host(X), host(Y))
    e = rel(host(g), g_ref)
    print(f"cfg5 N = {N}: loss rel {abs(loss - l_ref) / abs(l_ref):.2e}, grad rel {e:.2e}")
    assert abs(loss - l_ref) <= 1e-5 * abs(l_ref)
    assert e <= 1e-4


def test_cfg5_loss_grad_1m_route_matches_fp64(ctx, pkg, O):
    """cfg 5 at 32768 rows, the smallest N at which every GEMM of the N = 1,000,000 evaluation takes the 1M route's
    tile and split plan (LBF_SHOW_PLAN, profiles/r06/: dW layer 0 128 x 128 in 29 splits, layer 1 in 47, the last
    layer's forward on 128-row tiles; only the last layer's 1024 x 1 dW split count still grows with N). The fp64
    reference is torch CPU autograd on BLAS (O.torch_loss_grad; the C restatement is pinned to it at 1e-12 in
    tests/test_oracle.py and is too slow here). Loss 1e-5, gradient 1e-4."""
    dims, acts = CFG5
    N = 32768
    X, Y = pkg.synth_regression(ctx, N, dims[0])
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    loss, g = net.loss_grad(P, X, Y)
    l_ref, g_ref = O.torch_loss_grad(dims, acts, host(P), host(X), host(Y))
    e = rel(host(g), g_ref)
    print(f"cfg5 N = {N}: loss rel {abs(loss - l_ref) / abs(l_ref):.2e}, grad rel {e:.2e}")
    assert abs(loss - l_ref) <= 1e-5 * abs(l_ref)
    assert e <= 1e-4


def test_cfg5_lbfgs_m50_trajectory(ctx, pkg, O):
    dims, acts = CFG5
    N = 128
    X, Y = pkg.synth_regression(ctx, N, dims[0])
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    P0 = host(P)
    hist, _ = pkg.lbfgs_solve(net, P, X, Y, m=50, max_iters=6, tol=0.0)
    _, rec, _ = O.Net(dims, acts).lbfgs_wolfe(P0, host(X), host(Y), m=50, max_iters=6)
    r = np.abs(hist["loss"] - rec[:, 0]) / np.abs(rec[:, 0])
    assert r.max() <= 1e-3, r
    assert np.array_equal(hist["ls_trials"], rec[:, 4].astype(int))


def test_cfg5_full_size_properties(ctx, pkg):
    """N = 1,000,000 (16.4 GB of X in HBM): g.d equals the central difference of the loss, the sum of
    two half-batch shards scaled by 1/N equals the full-batch gradient (the all-reduce's algebra), and
    the m = 50 Wolfe iterations after the first decrease the loss (iteration 0 is the reference's blind
    step alpha = min(1, 1/||g||) without a line search, lbfgs.hpp:62-63, which here raises the loss)."""
    dims, acts = CFG5
    N = 1_000_000
    X, Y = pkg.synth_regression(ctx, N, dims[0])
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    loss, g = net.loss_grad(P, X, Y)
    d = torch.randn(P.numel(), device="cuda", generator=torch.Generator(device="cuda").manual_seed(0))
    d = d / d.norm()
    eps = 1e-2
    lp, _ = net.loss_grad(P + eps * d, X, Y)
    lm, _ = net.loss_grad(P - eps * d, X, Y)
    fd = (lp - lm) / (2 * eps)
    gd = float((g.double() * d.double()).sum())
    assert abs(fd - gd) <= 5e-3 * max(abs(gd), 1e-4), (fd, gd)
    h = N // 2
    l0, g0 = net.loss_grad(P, X[:h], Y[:h], inv_scale=1.0 / N)
    l1, g1 = net.loss_grad(P, X[h:], Y[h:], inv_scale=1.0 / N)
    assert abs((l0 + l1) - loss) <= 1e-6 * abs(loss)
    assert rel(host(g0) + host(g1), host(g)) <= 1e-5
    del g0, g1
    hist, info = pkg.lbfgs_solve(net, P, X, Y, m=50, max_iters=4, tol=0.0)
    assert len(hist["loss"]) == 4 and np.all(np.isfinite(hist["loss"]))
    assert np.all(np.diff(hist["loss"]) < 0)
    assert np.all(hist["accepted"][:3] == 1)
