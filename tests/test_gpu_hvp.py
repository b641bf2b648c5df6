"""Exact Hessian-vector product (R-operator, lbfgs-ffnn_amd/csrc/hvp.hip) vs
torch fp64 double-backward of the same loss (0.5 * inv_scale * ||net(X) - Y||^2 + 0.5 * lambda * ||w||^2,
the reference's batch_f / batch_g of unified_optimization.hpp:343-400) on the CPU.

Tolerance: ||Hv_gpu - Hv_ref|| / ||Hv_ref|| <= 1e-4 (fp32 products, fp64 reference). The S-LBFGS
option (hvp_exact) is checked for a descending run and against the finite-difference default.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

NETS = [
    ([20, 16, 3], ["tanh", "linear"]),
    ([30, 24, 12, 4], ["sigmoid", "relu", "linear"]),
    ([784, 128, 10], ["relu", "linear"]),
    ([64, 96, 33, 1], ["sigmoid", "tanh", "linear"]),
    ([40, 8], ["tanh"]),
    # output wider than every input: the R-forward's R{A} W product is B x out
    ([4, 6, 12], ["tanh", "linear"]),
    ([10, 5, 20], ["relu", "sigmoid"]),
]
ACTS = {"linear": lambda z: z, "relu": torch.relu, "tanh": torch.tanh, "sigmoid": torch.sigmoid}


def torch_loss(dims, acts, X, Y, inv_scale, lam):
    def f(P):
        a, off = X, 0
        for l in range(len(acts)):
            i, o = dims[l], dims[l + 1]
            W = P[off:off + i * o].reshape(i, o)
            b = P[off + i * o:off + (i + 1) * o]
            off += (i + 1) * o
            a = ACTS[acts[l]](a @ W + b)
        return 0.5 * inv_scale * ((a - Y) ** 2).sum() + 0.5 * lam * (P * P).sum()
    return f


@pytest.mark.parametrize("dims,acts", NETS)
@pytest.mark.parametrize("lam,gather", [(0.0, False), (1e-4, True)])
def test_hvp_matches_torch_fp64(ctx, pkg, dims, acts, lam, gather):
    rng = np.random.default_rng(len(dims) * 7 + dims[0])
    N = 37
    X = rng.standard_normal((N, dims[0])).astype(np.float32)
    Y = rng.standard_normal((N, dims[-1])).astype(np.float32)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    v = torch.from_numpy(rng.standard_normal(net.nparams).astype(np.float32)).cuda()
    idx = None
    rows = np.arange(N)
    if gather:
        rows = rng.permutation(N)[:23]
        idx = torch.from_numpy(rows.astype(np.int32)).cuda()
    B = len(rows)
    Xd, Yd = torch.from_numpy(X).cuda(), torch.from_numpy(Y).cuda()
    hv = net.hvp(P, v, Xd, Yd, idx=idx, inv_scale=1.0 / B, l2=lam)
    f = torch_loss(dims, acts, torch.from_numpy(X[rows]).double(), torch.from_numpy(Y[rows]).double(), 1.0 / B, lam)
    _, ref = torch.autograd.functional.hvp(f, P.double().cpu(), v.double().cpu())
    err = (hv.double().cpu() - ref).norm() / ref.norm()
    assert err <= 1e-4, float(err)


def test_hvp_linear_in_v_and_symmetric(ctx, pkg):
    """Size-independent properties at the cfg-2 shape, N = 4096: H(a u + b w) = a Hu + b Hw and
    w.Hu = u.Hw (the Hessian is symmetric)."""
    dims, acts = [784, 128, 10], ["relu", "linear"]
    Xh, Yh = pkg.synth_mnist(4096)
    X, Y = torch.from_numpy(Xh).cuda(), torch.from_numpy(Yh).cuda()
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    g = torch.Generator(device="cuda").manual_seed(1)
    u = torch.randn(net.nparams, device="cuda", generator=g)
    w = torch.randn(net.nparams, device="cuda", generator=g)
    Hu = net.hvp(P, u, X, Y).double()
    Hw = net.hvp(P, w, X, Y).double()
    Hc = net.hvp(P, 2.0 * u - 0.5 * w, X, Y).double()
    assert (Hc - (2.0 * Hu - 0.5 * Hw)).norm() <= 1e-5 * Hc.norm()
    a, b = float(w.double() @ Hu), float(u.double() @ Hw)
    assert abs(a - b) <= 1e-4 * max(abs(a), abs(b))


def test_hvp_dp_route_equals_single(ctx, pkg):
    dims, acts = [30, 24, 12, 4], ["sigmoid", "relu", "linear"]
    rng = np.random.default_rng(3)
    X = torch.from_numpy(rng.standard_normal((64, 30)).astype(np.float32)).cuda()
    Y = torch.from_numpy(rng.standard_normal((64, 4)).astype(np.float32)).cuda()
    c = pkg.Context(0)
    c.comm_init(1, 0, pkg.Context.unique_id())
    out = []
    for cc in (ctx, c):
        net = pkg.Mlp(cc, dims, acts)
        P = net.init_params(5, "cpu")
        v = torch.ones(net.nparams, device="cuda")
        out.append(net.hvp(P, v, X, Y, l2=1e-4).clone())
    assert torch.equal(out[0], out[1])


def test_slbfgs_exact_hvp_option(ctx, pkg):
    """S-LBFGS with the exact HVP (hvp_exact = 1) against the reference's finite-difference default:
    both descend, the curvature-pair counts agree and the losses stay within a few percent."""
    dims, acts = [784, 16, 10], ["relu", "linear"]
    Xh, Yh = pkg.synth_mnist(512)
    X, Y = torch.from_numpy(Xh).cuda(), torch.from_numpy(Yh).cuda()
    kw = dict(M=5, L=4, b=32, b_H=16, step=0.02, max_epochs=3, tol=0.0, lam=1e-4)
    res = {}
    for exact in (0, 1):
        net = pkg.Mlp(ctx, dims, acts)
        P = net.init_params(123, "cpu")
        hist, info = pkg.slbfgs_solve(net, P, X, Y, hvp_exact=exact, **kw)
        res[exact] = hist
    for h in res.values():
        assert np.all(np.isfinite(h["loss"])) and h["loss"][-1] < h["loss"][0]
    assert np.array_equal(res[0]["accepted"], res[1]["accepted"])
    r = np.abs(res[1]["loss"] - res[0]["loss"]) / np.abs(res[0]["loss"])
    assert r.max() <= 5e-2, r


def test_hvp_empty_batch(ctx, pkg):
    """A data-parallel rank's share of the b_H batch may be empty: H v is then the L2 term lambda v (and
    the rank still joins the all-reduce), not an error."""
    dims, acts = [30, 24, 4], ["tanh", "linear"]
    X = torch.zeros((1, 30), device="cuda")
    Y = torch.zeros((1, 4), device="cuda")
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(5, "cpu")
    v = torch.randn(net.nparams, device="cuda", generator=torch.Generator(device="cuda").manual_seed(2))
    idx = torch.zeros(0, dtype=torch.int32, device="cuda")
    hv = net.hvp(P, v, X, Y, idx=idx, inv_scale=1.0, l2=1e-4)
    ref = (1e-4 * v.double()).float()
    assert torch.allclose(hv, ref, rtol=1e-6, atol=0)


def test_fd_hvp_across_a_relu_kink_matches_oracle(ctx, pkg, O):
    """VERDICT r02 item 6, the step-0.01 NaN of config 4 (profiles/r03/diag_nan_step0.01.txt, diag_pair0.txt):
    the reference's finite-difference HVP (s_lbfgs.hpp:88-101) differences the gradient at u +- eps s; when
    a ReLU pre-activation changes sign in between, the gradient jumps and y picks up a term of order
    |jump| / (2 eps) the Hessian does not have. At cfg 4's first pair one sign flip in 32768 made |y| 20x the
    exact HVP's — in the device AND the fp64 / fp32 oracle alike at the same (u, s, rows); which run meets
    such a pair first is a knife edge of the trajectory. Here a kink is placed on purpose (one hidden unit's
    pre-activation is 0 at u on one row, and s moves it): the device FD equals the oracle's fp64 FD and both
    are far from the exact R-operator HVP, which is what a device bug could not produce."""
    dims, acts = [32, 16, 4], ["relu", "linear"]
    rng = np.random.default_rng(5)
    N, eps = 8, 1e-4
    X = rng.standard_normal((N, dims[0]))
    Y = rng.standard_normal((N, dims[-1]))
    net = pkg.Mlp(ctx, dims, acts)
    u = net.init_params(3, "cpu").double().cpu().numpy()
    n0 = dims[0] * dims[1]
    W0 = u[:n0].reshape(dims[0], dims[1])
    j = 5
    u[n0 + j] = -(X[0] @ W0[:, j])          # unit j of layer 0 sits exactly on its kink at row 0
    s = 0.01 * rng.standard_normal(u.size)
    s[n0 + j] = 1.0                         # ... and s crosses it: z = +-eps on that row
    # the fp32 copies both sides use (the oracle restates the device's fp32 inputs in fp64)
    u32, s32 = u.astype(np.float32), s.astype(np.float32)
    X32, Y32 = X.astype(np.float32), Y.astype(np.float32)
    onet = O.Net(dims, acts)
    rows = np.arange(N)
    y_or = onet.fd_hvp(u32.astype(np.float64), s32.astype(np.float64), X32.astype(np.float64),
                       Y32.astype(np.float64), idx=rows, lam=0.0, eps=eps)
    ud, sd = torch.from_numpy(u32).cuda(), torch.from_numpy(s32).cuda()
    Xd, Yd = torch.from_numpy(X32).cuda(), torch.from_numpy(Y32).cuda()
    y_fd = net.fd_hvp(ud, sd, Xd, Yd, inv_scale=1.0 / N, l2=0.0, eps=eps).double().cpu().numpy()
    y_ex = net.hvp(ud, sd, Xd, Yd, inv_scale=1.0 / N, l2=0.0).double().cpu().numpy()
    # the kink term: the FD result is far from the Hessian's product ...
    assert np.linalg.norm(y_fd - y_ex) > 0.5 * np.linalg.norm(y_ex)
    # ... and the device's FD is the reference algorithm's FD (fp32 differencing of fp32 gradients; the
    # fp64 oracle differences exact gradients: agreement to the fp32 gradient rounding / (2 eps))
    assert np.linalg.norm(y_fd - y_or) <= 2e-2 * np.linalg.norm(y_or), \
        (np.linalg.norm(y_fd - y_or) / np.linalg.norm(y_or))
