"""The EPI_HEAD fold (runtime.cpp Mlp::plan, head_core.hpp tile<.., FOLD>): the last hidden layer's
[dW ; db] rows past the dW GEMM's last full row tile (<= 16 input columns + the bias row) are
accumulated in the forward GEMM's epilogue instead of a mostly empty dW row tile.

Checked against the fp64 oracle (small N) and against the unfolded route (LBF_NO_FOLD=1, any N):
gradient relative difference <= 1e-4 / 2e-5 (fp32 products, different summation order).
Shapes: fold of 16 columns (784 = 6 x 128 + 16), 4 columns (260 = 2 x 128 + 4), the bias row
alone (In = 256), no fold (In % 4 != 0), hidden widths below / at the 128-column tile, both dW
tile heights (N <= 16384: 64-row tiles; larger N: 128-row tiles), gathered rows.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [
    ([784, 128, 10], ["relu", "linear"]),
    ([260, 96, 5], ["tanh", "sigmoid"]),
    ([256, 128, 10], ["sigmoid", "linear"]),
    ([144, 64, 3], ["relu", "tanh"]),
    ([130, 40, 7], ["relu", "linear"]),
    ([64, 784, 128, 10], ["tanh", "relu", "linear"]),
]


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def problem(dims, N, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((N, dims[0])).astype(np.float32)
    Y = rng.standard_normal((N, dims[-1])).astype(np.float32)
    return X, Y


def grads(pkg, ctx, dims, acts, X, Y, idx, monkeypatch, fold):
    if fold:
        monkeypatch.delenv("LBF_NO_FOLD", raising=False)
    else:
        monkeypatch.setenv("LBF_NO_FOLD", "1")
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(11, "cpu")
    loss, g = net.loss_grad(P, X, Y, idx=idx, l2=1e-4)
    return net, P, loss, g.double().cpu().numpy()


@pytest.mark.parametrize("dims,acts", SHAPES)
@pytest.mark.parametrize("N,gather", [(777, False), (777, True), (20000, False), (40000, True)])
def test_fold_equals_unfolded(ctx, pkg, monkeypatch, dims, acts, N, gather):
    Xh, Yh = problem(dims, N, seed=N + len(dims))
    X, Y = torch.from_numpy(Xh).cuda(), torch.from_numpy(Yh).cuda()
    idx = None
    if gather:
        rows = np.random.default_rng(5).permutation(N)[: N * 2 // 3].astype(np.int32)
        idx = torch.from_numpy(rows).cuda()
    _, _, l1, g1 = grads(pkg, ctx, dims, acts, X, Y, idx, monkeypatch, True)
    _, _, l0, g0 = grads(pkg, ctx, dims, acts, X, Y, idx, monkeypatch, False)
    assert abs(l1 - l0) <= 1e-6 * abs(l0)
    assert rel(g1, g0) <= 2e-5


@pytest.mark.parametrize("dims,acts", SHAPES[:4])
def test_fold_matches_oracle(ctx, pkg, O, monkeypatch, dims, acts):
    N = 517
    Xh, Yh = problem(dims, N, seed=3)
    net, P, loss, g = grads(pkg, ctx, dims, acts, torch.from_numpy(Xh).cuda(), torch.from_numpy(Yh).cuda(), None,
                            monkeypatch, True)
    l_ref, g_ref = O.Net(dims, acts).loss_grad(P.double().cpu().numpy(), Xh.astype(np.float64),
                                               Yh.astype(np.float64), lam=1e-4)
    assert abs(loss - l_ref) <= 1e-5 * abs(l_ref)
    assert rel(g, g_ref) <= 1e-4
