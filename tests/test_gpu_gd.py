"""GPU GD / SGD with momentum (CudaGD src/cuda/gd.cuh:38-106, CudaSGD
src/cuda/sgd.cuh:50-153) vs the oracle's fp32 restatement of the same loops (oracle/oracle.hpp
gd_momentum / sgd_momentum). The reference runs these in fp32 scalars, so the fp32 oracle is the
parity target; tolerance 1e-3 relative on the recorded losses (fp32 evaluation order differs), and
identical iteration counts where a stopping rule fires."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DIMS, ACTS = [784, 32, 10], ["relu", "linear"]


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()


def host(t):
    return t.double().cpu().numpy()


@pytest.mark.parametrize("momentum", [0.9, 0.0])
def test_gd_matches_oracle(ctx, pkg, O, momentum):
    Xh, Yh = pkg.synth_mnist(256)
    net = pkg.Mlp(ctx, DIMS, ACTS)
    P = net.init_params(123, "cuda")
    P0 = host(P)
    hist, info = pkg.gd_solve(net, P, dev(Xh), dev(Yh), lr=0.1, momentum=momentum, max_iters=15, tol=1e-6)
    Pr, rec = O.Net(DIMS, ACTS).gd(P0, Xh.astype(np.float64), Yh.astype(np.float64), lr=0.1, momentum=momentum,
                                   max_iters=15, tol=1e-6, fp32=True)
    assert info.iterations == len(rec) == 15
    r = np.abs(hist["loss"] - rec[:, 0]) / np.abs(rec[:, 0])
    assert r.max() <= 1e-3, r
    assert np.linalg.norm(host(P) - Pr) <= 1e-3 * np.linalg.norm(Pr)


def test_gd_tolerance_stop(ctx, pkg, O):
    """||g|| < tol ends the loop before the update (gd.cuh:73): same iteration count as the oracle."""
    Xh, Yh = pkg.synth_mnist(128)
    net = pkg.Mlp(ctx, DIMS, ACTS)
    P = net.init_params(123, "cuda")
    P0 = host(P)
    _, rec = O.Net(DIMS, ACTS).gd(P0, Xh.astype(np.float64), Yh.astype(np.float64), lr=0.1, momentum=0.9,
                                  max_iters=30, tol=1e-6, fp32=True)
    tol = float(rec[9, 1]) * (1 + 1e-3)  # between the norms recorded at iterations 9 and 10
    hist, info = pkg.gd_solve(net, P, dev(Xh), dev(Yh), lr=0.1, momentum=0.9, max_iters=30, tol=tol)
    _, rec2 = O.Net(DIMS, ACTS).gd(P0, Xh.astype(np.float64), Yh.astype(np.float64), lr=0.1, momentum=0.9,
                                   max_iters=30, tol=tol, fp32=True)
    assert info.iterations == len(rec2) < 30


@pytest.mark.parametrize("N,batch", [(256, 64), (250, 64)])
def test_sgd_matches_oracle(ctx, pkg, O, N, batch):
    """Contiguous batches (a ragged last batch for N = 250), momentum, step decay every 2 epochs."""
    Xh, Yh = pkg.synth_mnist(N)
    net = pkg.Mlp(ctx, DIMS, ACTS)
    P = net.init_params(123, "cuda")
    P0 = host(P)
    kw = dict(batch=batch, lr=0.05, momentum=0.9, decay_rate=0.5, decay_step=2, max_epochs=5, tol=0.0)
    hist, info = pkg.sgd_solve(net, P, dev(Xh), dev(Yh), **kw)
    Pr, rec = O.Net(DIMS, ACTS).sgd(P0, Xh.astype(np.float64), Yh.astype(np.float64), fp32=True, **kw)
    assert len(hist["loss"]) == len(rec) == 6
    r = np.abs(hist["loss"] - rec[:, 0]) / np.abs(rec[:, 0])
    assert r.max() <= 1e-3, r
    assert np.linalg.norm(host(P) - Pr) <= 1e-3 * np.linalg.norm(Pr)
    assert hist["alpha"][-1] == pytest.approx(0.05 * 0.25)   # decayed at epochs 2 and 4


def test_sgd_relative_improvement_stop(ctx, pkg, O):
    Xh, Yh = pkg.synth_mnist(256)
    net = pkg.Mlp(ctx, DIMS, ACTS)
    P = net.init_params(123, "cuda")
    P0 = host(P)
    kw = dict(batch=32, lr=0.01, momentum=0.0, max_epochs=40, tol=2e-2)
    hist, info = pkg.sgd_solve(net, P, dev(Xh), dev(Yh), **kw)
    _, rec = O.Net(DIMS, ACTS).sgd(P0, Xh.astype(np.float64), Yh.astype(np.float64), fp32=True, **kw)
    assert len(rec) < 41 and len(hist["loss"]) == len(rec)


def test_gd_dp_route_equals_single(ctx, pkg):
    Xh, Yh = pkg.synth_mnist(512)
    c = pkg.Context(0)
    c.comm_init(1, 0, pkg.Context.unique_id())
    out = []
    for cc in (ctx, c):
        net = pkg.Mlp(cc, DIMS, ACTS)
        P = net.init_params(7, "cuda")
        hist, _ = pkg.gd_solve(net, P, dev(Xh), dev(Yh), lr=0.1, momentum=0.9, max_iters=10, tol=0.0)
        out.append((hist["loss"], host(P)))
    assert np.allclose(out[0][0], out[1][0], rtol=1e-6, atol=0)
    assert np.array_equal(out[0][1], out[1][1])
