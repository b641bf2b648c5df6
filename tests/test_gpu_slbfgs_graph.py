"""S-LBFGS epochs replayed from captured hipGraphs (SlbfgsSolver::epoch_graph) against the eager route.

An epoch's launch sequence (s_lbfgs.hpp:218-262 inner steps: minibatch gradients, the fused direction,
the iterate update, the FD curvature pair every L steps) depends only on its batch slices, buffers and the
profiler's configuration, so from its second occurrence on the library captures it once (both streams:
the twin's anchor gradients fork and join through the same events) and replays it with one
hipGraphLaunch. Replays must be bitwise the eager epochs: same kernels, same arguments, same order on
each stream. Also the stateful API (lbf_slbfgs_begin / iterate / end) against one lbf_slbfgs_solve call,
and against the fp64 oracle over epochs that run from a graph.
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


def solve(pkg, ctx, Xh, Yh, monkeypatch, graph, anchor=0, epochs=6, chunks=None):
    monkeypatch.setenv("LBF_SLBFGS_GRAPH", "1" if graph else "0")
    monkeypatch.setenv("LBF_SLBFGS_ANCHOR", str(anchor))
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


@pytest.mark.parametrize("anchor", [0, 1])
def test_graph_epochs_equal_eager(ctx, pkg, monkeypatch, anchor):
    """6 epochs (LBF_SLBFGS_GRAPH=1): epoch 0 and 1 eager (first sight of each launch sequence), 2 captured,
    3-5 replayed."""
    Xh, Yh = pkg.synth_mnist(1024)
    Pg, lg, ag, ig = solve(pkg, ctx, Xh, Yh, monkeypatch, graph=True, anchor=anchor)
    Pe, le, ae, ie = solve(pkg, ctx, Xh, Yh, monkeypatch, graph=False, anchor=anchor)
    assert np.array_equal(Pg, Pe)
    assert np.array_equal(lg, le)
    assert np.array_equal(ag, ae)
    assert ig.n_evals == ie.n_evals and ig.n_rows == ie.n_rows  # replays count their evaluations
    assert np.all(np.isfinite(lg)) and lg[-1] < lg[0]


def test_stateful_run_equals_one_solve(ctx, pkg, monkeypatch):
    """begin / iterate(1) / iterate(2) / iterate(3) == one 6-epoch solve (same RNG stream, graphs reused
    across calls)."""
    Xh, Yh = pkg.synth_mnist(1024)
    Ps, ls, as_, _ = solve(pkg, ctx, Xh, Yh, monkeypatch, graph=True, chunks=[1, 2, 3])
    P1, l1, a1, _ = solve(pkg, ctx, Xh, Yh, monkeypatch, graph=True)
    assert np.array_equal(Ps, P1)
    assert np.array_equal(ls, l1)
    assert np.array_equal(as_, a1)


def test_graph_epochs_match_oracle(ctx, pkg, O, monkeypatch):
    """Epochs 2-4 come from a graph: the oracle's fp64 S-LBFGS (s_lbfgs.hpp:165-290) over the same draws."""
    dims, acts = [784, 16, 10], ["relu", "linear"]
    N = 512
    Xh, Yh = pkg.synth_mnist(N)
    monkeypatch.setenv("LBF_SLBFGS_GRAPH", "1")
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


def test_graph_profiler_times_replayed_launches(ctx, pkg, monkeypatch):
    """The bench's sampled section timing inside replayed epochs: event-record nodes of the graph, read
    after each replay; the same number of timed launches per epoch as an eager epoch."""
    Xh, Yh = pkg.synth_mnist(1024)
    counts = {}
    for graph in (False, True):
        monkeypatch.setenv("LBF_SLBFGS_GRAPH", "1" if graph else "0")
        net = pkg.Mlp(ctx, DIMS, ACTS)
        P = net.init_params(123, "cpu")
        run = pkg.SlbfgsRun(net, P, dev(Xh), dev(Yh), **KW)
        run.iterate(1)
        ctx.prof_select("gemm_fwd[0]")
        ctx.prof_sample(4)
        ctx.prof_enable(True)
        run.iterate(2)                 # eager, then captured
        ctx.prof_enable(True)          # clear
        run.iterate(3)                 # replayed (graph) / eager
        prof = ctx.prof_read()
        ctx.prof_enable(False)
        ctx.prof_select(None)
        ctx.prof_sample(1)
        run.close()
        ms, n = prof["gemm_fwd[0]"]
        assert n > 0 and ms > 0 and np.isfinite(ms)
        assert ms / n < 5.0  # milliseconds per launch: sane elapsed times, not garbage
        counts[graph] = n
    # the sampling phase is frozen in the graph (the capture epoch's), so the counts agree to a few launches
    assert abs(counts[True] - counts[False]) <= 3, counts


def test_in_launch_combine_matches_separate_launch(ctx, pkg, O, monkeypatch):
    """The S-LBFGS direction's linear combination inside the column-sum launch (dir.hip combine workers,
    s_lbfgs.hpp:218-262: r = H v, w_t -= step r; opt-in LBF_DIR_COMBINE=1) against the separate
    combine_small launch (the default): the same coefficients summed slot by slot instead of in logical order, so the
    iterates agree to fp64-summation rounding; also against the fp64 oracle."""
    dims, acts = [784, 16, 10], ["relu", "linear"]
    N = 512
    Xh, Yh = pkg.synth_mnist(N)
    kw = dict(M=5, L=4, b=32, b_H=16, step=0.02)
    out = {}
    for comb in ("1", "0"):
        monkeypatch.setenv("LBF_DIR_COMBINE", comb)
        net = pkg.Mlp(ctx, dims, acts)
        P = net.init_params(123, "cpu")
        P0 = host(P)
        hist, _ = pkg.slbfgs_solve(net, P, dev(Xh), dev(Yh), max_epochs=4, tol=0.0, lam=1e-4, **kw)
        out[comb] = (hist, host(P))
    (h1, P1), (h0, P0b) = out["1"], out["0"]
    assert np.array_equal(h1["accepted"], h0["accepted"])
    assert np.abs(h1["loss"] - h0["loss"]).max() <= 1e-6 * np.abs(h0["loss"]).max()
    assert np.abs(P1 - P0b).max() <= 1e-5 * np.abs(P0b).max()
    _, rec, _ = O.Net(dims, acts).slbfgs(P0, Xh.astype(np.float64), Yh.astype(np.float64), epochs=4, tol=0.0,
                                         M=5, L=4, b=32, bH=16, step=0.02, lam=1e-4)
    r = np.abs(h1["loss"] - rec[:, 0]) / np.abs(rec[:, 0])
    assert r.max() <= 1e-3, r
