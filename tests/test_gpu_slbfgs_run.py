"""The stateful S-LBFGS API (lbf_slbfgs_begin / iterate / end), which the benchmark drives: epochs split over
several iterate() calls are bitwise one lbf_slbfgs_solve (same RNG stream, the next epoch's draws made while
the current one runs), they match the fp64 oracle's S-LBFGS (s_lbfgs.hpp:165-290) over the same draws, and the
profiler's sampled section timing covers the twin stream's launches.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()


def host(t):
    return t.double().cpu().numpy()


DIMS, ACTS = [784, 64, 10], ["relu", "linear"]
KW = dict(M=5, L=4, b=64, b_H=32, step=0.01, lam=1e-4, tol=0.0)


def solve(pkg, ctx, Xh, Yh, epochs=6, chunks=None):
    net = pkg.Mlp(ctx, DIMS, ACTS)
    P = net.init_params(123, "cpu")
    X, Y = dev(Xh), dev(Yh)
    if chunks is None:
        hist, info = pkg.slbfgs_solve(net, P, X, Y, max_epochs=epochs, **KW)
        return host(P), hist["loss"], hist["accepted"], info
    run = pkg.SlbfgsRun(net, P, X, Y, **KW)
    for c in chunks:
        run.iterate(c)
    torch.cuda.synchronize()
    out = host(P), run.hist.as_dict()["loss"], run.hist.as_dict()["accepted"], run.info
    run.close()
    return out


def test_stateful_run_equals_one_solve(ctx, pkg):
    """begin / iterate(1) / iterate(2) / iterate(3) == one 6-epoch solve."""
    Xh, Yh = pkg.synth_mnist(1024)
    Ps, ls, as_, is_ = solve(pkg, ctx, Xh, Yh, chunks=[1, 2, 3])
    P1, l1, a1, i1 = solve(pkg, ctx, Xh, Yh)
    assert np.array_equal(Ps, P1)
    assert np.array_equal(ls, l1)
    assert np.array_equal(as_, a1)
    assert is_.n_evals == i1.n_evals and is_.n_rows == i1.n_rows
    assert np.all(np.isfinite(l1)) and l1[-1] < l1[0]


def test_multi_epoch_matches_oracle(ctx, pkg, O):
    """Five epochs against the oracle's fp64 S-LBFGS over the same draws."""
    dims, acts = [784, 16, 10], ["relu", "linear"]
    N = 512
    Xh, Yh = pkg.synth_mnist(N)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    P0 = host(P)
    kw = dict(M=5, L=4, b=32, b_H=16, step=0.02)
    hist, _ = pkg.slbfgs_solve(net, P, dev(Xh), dev(Yh), max_epochs=5, tol=0.0, lam=1e-4, **kw)
    _, rec, _ = O.Net(dims, acts).slbfgs(P0, Xh.astype(np.float64), Yh.astype(np.float64), epochs=5, tol=0.0,
                                         M=5, L=4, b=32, bH=16, step=0.02, lam=1e-4)
    r = np.abs(hist["loss"] - rec[:, 0]) / np.abs(rec[:, 0])
    assert r.max() <= 1e-3, r
    assert np.array_equal(hist["accepted"], rec[:, 3].astype(int))


def test_profiler_times_sampled_launches(ctx, pkg):
    """The bench's sampled section timing over S-LBFGS epochs (context and twin streams): sane elapsed times
    and the expected number of timed launches."""
    Xh, Yh = pkg.synth_mnist(1024)
    net = pkg.Mlp(ctx, DIMS, ACTS)
    P = net.init_params(123, "cpu")
    run = pkg.SlbfgsRun(net, P, dev(Xh), dev(Yh), **KW)
    run.iterate(1)
    ctx.prof_select("gemm_fwd[0]")
    ctx.prof_sample(1)
    ctx.prof_enable(True)
    run.iterate(2)
    prof = ctx.prof_read()
    ctx.prof_enable(False)
    ctx.prof_select(None)
    run.close()
    ms, n = prof["gemm_fwd[0]"]
    assert ms > 0 and np.isfinite(ms)
    assert ms / n < 5.0  # milliseconds per launch: sane elapsed times, not garbage
    # per epoch: 2 minibatch evaluations per inner step (w_t and the anchor on the twin), the FD pairs, the
    # full-batch gradient; 1024 / 64 = 16 inner steps
    assert 2 * 2 * 16 <= n <= 2 * (2 * 16 + 2 * 4 + 2), n


@pytest.mark.parametrize("L,N", [(4, 1024), (10, 640)])
def test_full_ahead_equals_ordered(ctx, pkg, monkeypatch, L, N):
    """The epoch-end full-batch evaluation at the picked anchor, started on a third stream once that iterate
    exists (SlbfgsSolver::post_full, opt-in LBF_FULL_AHEAD=1), is bitwise the ordered evaluation after the last
    inner step: losses, gradient norms, live pairs and parameters over several epochs, picks early
    and late in the ring (N = 640, b = 64: 10 inner steps, the whole epoch fits the L + 1 = 11 ring, so a pick
    of entry 0 is the epoch's own anchor, posted before the first step)."""
    Xh, Yh = pkg.synth_mnist(N)
    X, Y = dev(Xh), dev(Yh)
    kw = dict(KW, L=L)
    out = []
    for on in ("1", "0"):
        monkeypatch.setenv("LBF_FULL_AHEAD", on)
        net = pkg.Mlp(ctx, DIMS, ACTS)
        P = net.init_params(123, "cpu")
        hist, info = pkg.slbfgs_solve(net, P, X, Y, max_epochs=6, **kw)
        out.append((host(P), hist, info))
    (P0, h0, i0), (P1, h1, i1) = out
    assert np.array_equal(P0, P1)
    for k in ("loss", "grad_norm", "accepted"):
        assert np.array_equal(h0[k], h1[k]), k
    assert i0.n_evals == i1.n_evals and i0.n_rows == i1.n_rows
    assert np.all(np.isfinite(h0["loss"]))
