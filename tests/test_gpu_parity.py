"""GPU parity: HIP kernels (through the C ABI) vs the CPU oracle (fp64 restatement of the reference).

Tolerances (fp32 compute vs fp64 reference):
  loss: relative 1e-5; gradient: ||dg|| / ||g|| <= 1e-4; two-loop direction: ||dp|| / ||p|| <= 1e-5;
  L-BFGS trajectory (Wolfe, CPU semantics): first 10 iterations' loss relative <= 1e-3.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

LOSS_RTOL = 1e-5
GRAD_RTOL = 1e-4
DIR_RTOL = 1e-5


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()


def host(t):
    return t.double().cpu().numpy()


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def random_problem(dims, N, seed=0, onehot=True):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((N, dims[0])).astype(np.float32).astype(np.float64)
    if onehot:
        Y = np.zeros((N, dims[-1]))
        Y[np.arange(N), rng.integers(0, dims[-1], N)] = 1.0
    else:
        Y = rng.standard_normal((N, dims[-1])).astype(np.float32).astype(np.float64)
    return X, Y


NETS = [
    ([784, 128, 10], ["relu", "linear"]),
    ([784, 128, 64, 10], ["relu", "relu", "linear"]),
    ([37, 50, 3], ["tanh", "sigmoid"]),
    ([64, 96, 33, 1], ["sigmoid", "tanh", "linear"]),
    ([129, 130, 65, 10], ["relu", "tanh", "linear"]),
    # generic output path (no fused head): Out > 16, hidden > 256, single layer
    ([784, 300, 20], ["relu", "linear"]),
    ([16, 300, 4], ["tanh", "linear"]),
    ([50, 7], ["sigmoid"]),
]


@pytest.mark.parametrize("dims,acts", NETS)
@pytest.mark.parametrize("N", [1, 31, 257, 1000])
def test_loss_grad_matches_oracle(ctx, pkg, O, dims, acts, N):
    X, Y = random_problem(dims, N, seed=N)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    loss, g = net.loss_grad(P, dev(X), dev(Y))
    onet = O.Net(dims, acts)
    l_ref, g_ref = onet.loss_grad(host(P), X, Y)
    assert abs(loss - l_ref) <= LOSS_RTOL * abs(l_ref)
    # Tolerance = max(1e-4, 3x the rounding error of the reference algorithm itself run in fp32, i.e.
    # the oracle's fp32 instantiation vs fp64): some shapes cancel heavily (784-300-20 on N(0,1)
    # inputs loses ~4e-4 in ANY fp32 evaluation; the HIP result agrees with the fp32 oracle there).
    _, g32 = onet.loss_grad_f32(host(P), X, Y)
    assert rel(host(g), g_ref) <= max(GRAD_RTOL, 3.0 * rel(g32, g_ref))


def test_forward_matches_oracle(ctx, pkg, O):
    dims, acts = [784, 128, 10], ["relu", "linear"]
    X, Y = random_problem(dims, 300, seed=3)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(7, "cuda")
    out = host(net.forward(P, dev(X)))
    _, out_ref = O.Net(dims, acts).loss(host(P), X, Y, want_out=True)
    assert rel(out, out_ref) <= 1e-5


def test_loss_grad_gather_and_l2(ctx, pkg, O):
    """S-LBFGS batch_g: gathered minibatch rows + L2 term (unified_optimization.hpp:343-376)."""
    dims, acts = [784, 64, 10], ["relu", "linear"]
    Xh, Yh = pkg.synth_mnist(500)
    idx = O.sample_indices(500, 77, seed=123, calls=1)[0]
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    loss, g = net.loss_grad(P, dev(Xh), dev(Yh), idx=torch.from_numpy(idx.astype(np.int32)).cuda(), l2=1e-4)
    l_ref, g_ref = O.Net(dims, acts).loss_grad(host(P), Xh.astype(np.float64), Yh.astype(np.float64), idx=idx,
                                               lam=1e-4)
    assert abs(loss - l_ref) <= LOSS_RTOL * abs(l_ref)
    assert rel(host(g), g_ref) <= GRAD_RTOL


@pytest.mark.parametrize("dims,acts", [([784, 128, 10], ["relu", "linear"]),
                                       ([784, 128, 64, 10], ["relu", "relu", "linear"])])
@pytest.mark.parametrize("N,gather", [(8192, False), (8200, False), (15000, True), (30000, False),
                                      (32768, False), (32800, True)])
def test_forward_tile_routes_match_oracle(ctx, pkg, O, dims, acts, N, gather):
    """Mlp::plan's forward row tiles at a rank's shard sizes (its cost model picks 32 x 128 at 8192 rows,
    64 x 128 at 8200 / 15000 / 30000 / 32768 / 32800 on 256 CUs; 128 x 128 at 60000 elsewhere); each with
    the fused head and the fold, against the oracle (gathered rows: the S-LBFGS anchor path)."""
    Xh, Yh = pkg.synth_mnist(N, dims[0], dims[-1], 7)
    idx = np.random.default_rng(N).permutation(N)[: N - 37].astype(np.int64) if gather else None
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    loss, g = net.loss_grad(P, dev(Xh), dev(Yh),
                            idx=torch.from_numpy(idx.astype(np.int32)).cuda() if gather else None)
    l_ref, g_ref = O.Net(dims, acts).loss_grad(host(P), Xh.astype(np.float64), Yh.astype(np.float64), idx=idx)
    assert abs(loss - l_ref) <= LOSS_RTOL * abs(l_ref)
    assert rel(host(g), g_ref) <= GRAD_RTOL


@pytest.mark.parametrize("H", [132, 200, 255, 256])
@pytest.mark.parametrize("N", [1, 63, 256, 40000])
def test_standalone_head_matches_oracle(ctx, pkg, O, H, N):
    """The standalone head kernel (last hidden layer wider than 128, so not fused into its GEMM): tiles
    and W prefetched in registers (H % 4 == 0) or the scalar staging path (H = 255); at N = 40000 each
    workgroup walks two 64-row tiles, the second prefetched during the first."""
    dims, acts = [48, H, 10], ["relu", "linear"]
    X, Y = random_problem(dims, N, seed=H + N)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    loss, g = net.loss_grad(P, dev(X), dev(Y))
    onet = O.Net(dims, acts)
    l_ref, g_ref = onet.loss_grad(host(P), X, Y)
    assert abs(loss - l_ref) <= LOSS_RTOL * abs(l_ref)
    assert rel(host(g), g_ref) <= GRAD_RTOL


def test_eval_is_deterministic(ctx, pkg):
    """Fixed-order reductions: two evaluations of the same point are bitwise identical (the Wolfe
    line search's cached f / grad reuse relies on it)."""
    dims, acts = [784, 128, 10], ["relu", "linear"]
    Xh, Yh = pkg.synth_mnist(4096)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    X, Y = dev(Xh), dev(Yh)
    l1, g1 = net.loss_grad(P, X, Y)
    l2, g2 = net.loss_grad(P, X, Y)
    assert l1 == l2
    assert torch.equal(g1, g2)


def make_history(n, k, seed=0):
    rng = np.random.default_rng(seed)
    d = rng.uniform(0.5, 2.0, n)
    S = rng.standard_normal((k, n))
    Yv = S * d + 0.01 * rng.standard_normal((k, n))   # positive curvature pairs
    S = S.astype(np.float32).astype(np.float64)
    Yv = Yv.astype(np.float32).astype(np.float64)
    rho = 1.0 / np.einsum("ij,ij->i", S, Yv)
    g = rng.standard_normal(n).astype(np.float32).astype(np.float64)
    return S, Yv, rho, g


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("k", [0, 1, 5, 10, 30, 50, 70, 100, 128])
@pytest.mark.parametrize("n", [1000, 100003])
def test_two_loop_matches_oracle(ctx, O, mode, k, n):
    """k = 30 / 70 / 100 (m = k): SY with an odd row stride and YY's lower triangle in LDS, two indices
    per lane (the m = 100 history step); k = 128 is the largest history (global YY reads)."""
    S, Yv, rho, g = make_history(n, k, seed=k + n)
    ref = O.two_loop(mode, S if k else np.zeros((0, n)), Yv if k else np.zeros((0, n)), rho, g)
    out = ctx.two_loop(dev(S) if k else None, dev(Yv) if k else None, rho, dev(g), mode=mode)
    assert rel(host(out), ref) <= DIR_RTOL


@pytest.mark.parametrize("k", [1, 2, 5, 10, 16])
@pytest.mark.parametrize("near", [False, True], ids=["plain", "ys_near_threshold"])
def test_two_loop_kmat_route_matches_recurrences(ctx, O, k, near):
    """The S-LBFGS solver's direction-only step takes its coefficients from the map K that the last pair update
    built (compact form, an explicit R^-1; dir_combine_kernel), not from the two-loop recurrences. The same ring
    through that route (lbf_two_loop mode 3: each pair offered through the solver's pair update, then one
    direction-only step) against the recurrences (mode 1, dir_fin / hist_core) and the fp64 oracle's two-loop of
    s_lbfgs.hpp:106-136, at every live count the route supports; `ys_near_threshold` makes one middle pair's
    y.s = 3e-10, just above the acceptance threshold |y.s| > 1e-10 (s_lbfgs.hpp:245-256), so rho = 3.3e9 enters
    R^-1. The route also checks that K was built for the ring's live count (SC_KERR)."""
    n = 100000
    S, Yv, rho, g = make_history(n, k, seed=3 * k + int(near))
    if near:
        j = k // 2
        Yv[j] = (Yv[j] * (3e-10 / float(S[j] @ Yv[j]))).astype(np.float32).astype(np.float64)
        rho = 1.0 / np.einsum("ij,ij->i", S, Yv)
        assert 1e-10 < 1.0 / rho[j] < 1e-9
    ref = O.two_loop(1, S, Yv, rho, g)
    out1 = ctx.two_loop(dev(S), dev(Yv), rho, dev(g), mode=1)
    out3 = ctx.two_loop(dev(S), dev(Yv), rho, dev(g), mode=3)
    e31, e3, e1 = rel(host(out3), host(out1)), rel(host(out3), ref), rel(host(out1), ref)
    print(f"k {k} near {near}: K route vs recurrences {e31:.2e}, vs oracle {e3:.2e} (recurrences {e1:.2e})")
    assert e3 <= DIR_RTOL and e1 <= DIR_RTOL
    assert e31 <= DIR_RTOL


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("k", [5, 48])
def test_two_loop_large_n(ctx, O, mode, k):
    """n past 2M: the Gram sweep's chunks are longer than one pass of its loads (4096 elements per
    workgroup at cfg 5's n), and the history loads switch to nontemporal past the Infinity Cache."""
    n = 3_000_001
    S, Yv, rho, g = make_history(n, k, seed=k + 7)
    ref = O.two_loop(mode, S, Yv, rho, g)
    out = ctx.two_loop(dev(S), dev(Yv), rho, dev(g), mode=mode)
    assert rel(host(out), ref) <= DIR_RTOL


def test_blas1(ctx):
    rng = np.random.default_rng(1)
    x = rng.standard_normal(123457).astype(np.float32)
    y = rng.standard_normal(123457).astype(np.float32)
    dx, dy = dev(x), dev(y)
    assert abs(ctx.dot(dx, dy) - float(np.dot(x.astype(np.float64), y))) < 1e-9 * 123457
    assert abs(ctx.nrm2(dx) - float(np.linalg.norm(x.astype(np.float64)))) < 1e-9 * 400
    ctx.axpy_(0.5, dx, dy)
    assert np.allclose(host(dy), y + np.float32(0.5) * x, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("m", [5, 10])
def test_lbfgs_wolfe_trajectory(ctx, pkg, O, m):
    """CPU semantics (lbfgs.hpp:38-100 + full_batch_minimizer.hpp:126-157): fp32 GPU trajectory vs the
    fp64 oracle, same seed/data. Early iterations agree to 1e-3; the line-search decisions match."""
    dims, acts = [784, 32, 10], ["relu", "linear"]
    Xh, Yh = pkg.synth_mnist(256)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    P0 = host(P)
    hist, info = pkg.lbfgs_solve(net, P, dev(Xh), dev(Yh), m=m, max_iters=20, tol=0.0)
    _, rec, _ = O.Net(dims, acts).lbfgs_wolfe(P0, Xh.astype(np.float64), Yh.astype(np.float64), m=m,
                                              max_iters=20)
    assert len(hist["loss"]) == 20
    r = np.abs(hist["loss"][:10] - rec[:10, 0]) / np.abs(rec[:10, 0])
    assert r.max() <= 1e-3, r
    assert np.array_equal(hist["ls_trials"][:10], rec[:10, 4].astype(int))
    assert np.array_equal(hist["accepted"][:9], rec[:9, 3].astype(int))
    # monotone decrease (Armijo condition) on the whole run
    assert np.all(np.diff(hist["loss"]) <= 1e-7)


@pytest.mark.parametrize("line_search", ["wolfe", "armijo"])
def test_gram_fin_route_matches_oracle(ctx, pkg, O, monkeypatch, line_search):
    """m = 40 > TAIL_MAXM: every direction takes the unfused history path (lbfgs.hpp:106-139 /
    lbfgs.cuh:206-261), whose Gram partials are now summed per column by a launch whose last block runs
    the history step (gram_fin). Against the oracle, and against the fold_rows + hist_step route it
    replaces (LBF_GRAM_FIN=0): same line-search decisions, losses within fp64-summation-order rounding."""
    dims, acts = [784, 32, 10], ["relu", "linear"]
    Xh, Yh = pkg.synth_mnist(256)
    runs = {}
    for fin in ("1", "0"):
        monkeypatch.setenv("LBF_GRAM_FIN", fin)
        net = pkg.Mlp(ctx, dims, acts)
        P = net.init_params(123, "cpu" if line_search == "wolfe" else "cuda")
        P0 = host(P)
        runs[fin] = pkg.lbfgs_solve(net, P, dev(Xh), dev(Yh), line_search=line_search, m=40, max_iters=25,
                                    tol=0.0)[0]
    net_o = O.Net(dims, acts)
    if line_search == "wolfe":
        _, rec, _ = net_o.lbfgs_wolfe(P0, Xh.astype(np.float64), Yh.astype(np.float64), m=40, max_iters=25)
    else:
        _, rec = net_o.lbfgs_armijo(P0, Xh.astype(np.float64), Yh.astype(np.float64), m=40, max_iters=25,
                                    fp32=True)
    a, b = runs["1"], runs["0"]
    assert np.array_equal(a["ls_trials"][:15], b["ls_trials"][:15])
    assert np.abs(a["loss"][:15] - b["loss"][:15]).max() <= 1e-5 * np.abs(b["loss"][:15]).max()
    r = np.abs(a["loss"][:10] - rec[:10, 0]) / np.abs(rec[:10, 0])
    assert r.max() <= 1e-3, r
    assert np.array_equal(a["ls_trials"][:8], rec[:8, 4].astype(int))


def test_lbfgs_armijo_trajectory(ctx, pkg, O):
    """CUDA semantics (lbfgs.cuh:39-194) vs the oracle's fp32 instantiation of the same algorithm."""
    dims, acts = [784, 32, 10], ["relu", "linear"]
    Xh, Yh = pkg.synth_mnist(256)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cuda")
    P0 = host(P)
    hist, info = pkg.lbfgs_solve(net, P, dev(Xh), dev(Yh), line_search="armijo", m=10, max_iters=15, tol=0.0)
    _, rec = O.Net(dims, acts).lbfgs_armijo(P0, Xh.astype(np.float64), Yh.astype(np.float64), m=10,
                                            max_iters=15, fp32=True)
    r = np.abs(hist["loss"][:8] - rec[:8, 0]) / np.abs(rec[:8, 0])
    assert r.max() <= 1e-3, r
    assert np.array_equal(hist["ls_trials"][:8], rec[:8, 4].astype(int))


@pytest.mark.parametrize("case", [([4, 8, 2], ["tanh", "tanh"], 23), ([5, 5, 5, 2], ["tanh", "tanh", "tanh"], 15)],
                         ids=["4-8-2", "5-5-5-2"])
def test_lbfgs_armijo_rejected_pair_full_ring(ctx, pkg, O, case):
    """CUDA semantics with a full ring and a rejected pair (lbfgs.cuh:149-169: the oldest slot is overwritten
    in place, its rho left stale, and stays live): the history step's live Gram block then takes that slot's
    row and column from the fresh dots at its old index. Smooth tanh nets on 16 rows whose fp32 oracle rejects
    a pair at iteration 3-4 with m = 3 (found by a search over seeds); the device follows it through the
    rejection: same accept / reject record, same line-search trials, losses within 1e-3."""
    dims, acts, seed = case
    rng = np.random.default_rng(seed)
    Xh = rng.standard_normal((16, dims[0])).astype(np.float32)
    Yh = rng.standard_normal((16, dims[-1])).astype(np.float32)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(seed + 1, "cuda")
    P0 = host(P)
    hist, _ = pkg.lbfgs_solve(net, P, dev(Xh), dev(Yh), line_search="armijo", m=3, max_iters=12, tol=0.0)
    _, rec = O.Net(dims, acts).lbfgs_armijo(P0, Xh.astype(np.float64), Yh.astype(np.float64), m=3, max_iters=12,
                                            fp32=True)
    acc_ref = rec[:, 3].astype(int)
    assert (acc_ref[3:8] == 0).any(), "the case must reject a pair with the ring full"
    assert np.array_equal(hist["accepted"][:10], acc_ref[:10]), (hist["accepted"][:10], acc_ref[:10])
    assert np.array_equal(hist["ls_trials"][:10], rec[:10, 4].astype(int))
    r = np.abs(hist["loss"][:10] - rec[:10, 0]) / np.abs(rec[:10, 0])
    assert r.max() <= 1e-3, r


def test_slbfgs_matches_oracle(ctx, pkg, O):
    """S-LBFGS (s_lbfgs.hpp:165-290): same host RNG stream, same sampled batches, same curvature pairs."""
    dims, acts = [784, 16, 10], ["relu", "linear"]
    N = 512
    Xh, Yh = pkg.synth_mnist(N)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    P0 = host(P)
    kw = dict(M=5, L=4, b=32, b_H=16, step=0.02)
    hist, info = pkg.slbfgs_solve(net, P, dev(Xh), dev(Yh), max_epochs=2, tol=0.0, lam=1e-4, **kw)
    _, rec, _ = O.Net(dims, acts).slbfgs(P0, Xh.astype(np.float64), Yh.astype(np.float64), epochs=2, tol=0.0,
                                         M=5, L=4, b=32, bH=16, step=0.02, lam=1e-4)
    assert len(hist["loss"]) == 2
    r = np.abs(hist["loss"] - rec[:, 0]) / np.abs(rec[:, 0])
    assert r.max() <= 1e-3, r
    assert np.array_equal(hist["accepted"], rec[:, 3].astype(int))   # live pairs after each epoch


def test_gradient_directional_derivative_full_size(ctx, pkg):
    """Size-independent property at the BASELINE cfg-2 size (N = 60000): central difference of the loss
    along a random direction equals g.d (no oracle needed at full size)."""
    dims, acts = [784, 128, 10], ["relu", "linear"]
    Xh, Yh = pkg.synth_mnist(60000)
    X, Y = dev(Xh), dev(Yh)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    loss, g = net.loss_grad(P, X, Y)
    d = torch.randn_like(P, generator=torch.Generator(device="cuda").manual_seed(0))
    d = d / d.norm()
    eps = 1e-2
    lp, _ = net.loss_grad(P + eps * d, X, Y)
    lm, _ = net.loss_grad(P - eps * d, X, Y)
    fd = (lp - lm) / (2 * eps)
    gd = float((g.double() * d.double()).sum())
    assert abs(fd - gd) <= 2e-3 * max(abs(gd), 1e-3), (fd, gd)


def test_shard_sum_equals_full_batch(ctx, pkg):
    """Data-parallel decomposition at full size: sum of per-shard gradients scaled by 1/N_global equals
    the full-batch gradient (what the RCCL all-reduce computes)."""
    dims, acts = [784, 128, 10], ["relu", "linear"]
    Xh, Yh = pkg.synth_mnist(60000)
    X, Y = dev(Xh), dev(Yh)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    lf, gf = net.loss_grad(P, X, Y)
    gs = torch.zeros_like(gf, dtype=torch.float64)
    ls = 0.0
    for r in range(8):
        lo, hi = 60000 * r // 8, 60000 * (r + 1) // 8
        l, g = net.loss_grad(P, X[lo:hi].contiguous(), Y[lo:hi].contiguous(), inv_scale=1.0 / 60000)
        gs += g.double()
        ls += l
    assert abs(ls - lf) <= 1e-6 * abs(lf)
    assert rel(gs.cpu().numpy(), host(gf)) <= 1e-5


def test_lbfgs_full_size_decreases(ctx, pkg):
    """cfg 2 (784-128-10, N=60000, m=10): 10 Wolfe iterations run and decrease the loss monotonically."""
    dims, acts = [784, 128, 10], ["relu", "linear"]
    Xh, Yh = pkg.synth_mnist(60000)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    hist, info = pkg.lbfgs_solve(net, P, dev(Xh), dev(Yh), m=10, max_iters=10, tol=0.0)
    assert len(hist["loss"]) == 10
    assert np.all(np.diff(hist["loss"]) <= 0)
    assert hist["loss"][-1] < 0.5 * hist["loss"][0]


def _spec_run(pkg, ctx, monkeypatch, depth, line_search, tol, iters, chunks=1, fused=True, m=5):
    monkeypatch.setenv("LBF_SPEC_DEPTH", str(depth))
    monkeypatch.setenv("LBF_FUSED_TAIL", "1" if fused else "0")
    dims, acts = [784, 32, 10], ["relu", "linear"]
    Xh, Yh = pkg.synth_mnist(256)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(7, "cuda" if line_search == "armijo" else "cpu")
    run = pkg.LbfgsRun(net, P, dev(Xh), dev(Yh), line_search=line_search, m=m, max_iters=iters, tol=tol)
    for c in range(chunks):
        run.iterate(iters // chunks)
    info = run.info
    h = run.hist.as_dict()
    run.close()
    return h, (info.iterations, info.n_evals, info.final_loss, info.final_grad_norm, info.n_loss_only), host(P)


def _same(h, ref, keys=("loss", "grad_norm", "alpha", "ls_trials", "accepted")):
    return all(np.array_equal(h[k], ref[k]) for k in keys)


@pytest.mark.parametrize("line_search", ["wolfe", "armijo"])
def test_speculative_line_search_is_exact(ctx, pkg, monkeypatch, line_search):
    """Speculation (ls_ctl + abort flag, solvers.cpp iterate_spec) without the fused tail reproduces
    the host-driven loop bit for bit: records, evaluation count, final parameters — across rejections
    of the first trial, convergence inside the speculation window, and split iterate() calls."""
    ref, ref_info, ref_P = _spec_run(pkg, ctx, monkeypatch, 0, line_search, 0.0, 40)
    assert np.any(ref["ls_trials"][1:] > 1), "problem must exercise rejected first trials"
    for depth, chunks in [(1, 1), (3, 1), (8, 1), (3, 4)]:
        h, info, P = _spec_run(pkg, ctx, monkeypatch, depth, line_search, 0.0, 40, chunks, fused=False)
        assert _same(h, ref), (depth, chunks)
        assert info == ref_info, (depth, info, ref_info)
        assert np.array_equal(P, ref_P)
    tol = float(ref["grad_norm"][12]) * (1 + 1e-6)
    ref_c, ref_ci, ref_cP = _spec_run(pkg, ctx, monkeypatch, 0, line_search, tol, 40)
    assert len(ref_c["loss"]) < 40
    h, info, P = _spec_run(pkg, ctx, monkeypatch, 4, line_search, tol, 40, fused=False)
    assert info == ref_ci
    assert np.array_equal(h["loss"], ref_c["loss"]) and np.array_equal(P, ref_cP)


@pytest.mark.parametrize("line_search", ["wolfe", "armijo"])
@pytest.mark.parametrize("m", [5, 20])
def test_fused_tail_matches_host_loop(ctx, pkg, monkeypatch, line_search, m):
    """Fused optimizer tail (tail.hip): identical at every speculation depth and split of iterate();
    against the host-driven loop the only difference is the fp64 summation order of the Gram dots, so
    the line-search decisions are the same and the losses agree to 1e-9 relative (and a first trial
    rejected early, EarlyLs, is counted as the loss-only trial it was)."""
    ref, ref_info, ref_P = _spec_run(pkg, ctx, monkeypatch, 0, line_search, 0.0, 30, m=m)
    base, base_info, base_P = _spec_run(pkg, ctx, monkeypatch, 1, line_search, 0.0, 30, m=m)
    for depth, chunks in [(3, 1), (8, 1), (3, 5)]:
        h, info, P = _spec_run(pkg, ctx, monkeypatch, depth, line_search, 0.0, 30, chunks, m=m)
        assert _same(h, base), (depth, chunks)
        assert info == base_info and np.array_equal(P, base_P)
    assert np.array_equal(base["ls_trials"], ref["ls_trials"])
    assert np.array_equal(base["accepted"], ref["accepted"])
    # a first trial that fails sufficient decrease in its first backward GEMM (EarlyLs, fused route only) runs
    # its forward alone: one evaluation fewer and one loss-only trial more than the host loop's full evaluation
    assert base_info[0] == ref_info[0] and base_info[1] + base_info[4] == ref_info[1] + ref_info[4]
    assert base_info[1] <= ref_info[1]
    r = np.abs(base["loss"] - ref["loss"]) / np.abs(ref["loss"])
    assert r.max() <= 1e-9, r
    assert rel(base_P, ref_P) <= 1e-6
    # convergence inside the speculation window
    tol = float(ref["grad_norm"][12]) * (1 + 1e-6)
    ref_c, ref_ci, _ = _spec_run(pkg, ctx, monkeypatch, 0, line_search, tol, 30, m=m)
    h, info, _ = _spec_run(pkg, ctx, monkeypatch, 4, line_search, tol, 30, m=m)
    assert info[0] == ref_ci[0] and info[1] + info[4] == ref_ci[1] + ref_ci[4]
    assert np.allclose(h["loss"], ref_c["loss"], rtol=1e-9, atol=0)


@pytest.mark.parametrize("dims,acts", NETS[:6])
@pytest.mark.parametrize("N", [257, 20000])
def test_loss_only_equals_fused_loss(ctx, pkg, O, dims, acts, N):
    """lbf_mlp_loss (forward + MSE, a line-search trial's f) reports bitwise the loss of the full
    evaluation of the same point (same SSE partials, same reduction order): the Wolfe / Armijo decisions
    taken on it are the full evaluation's."""
    X, Y = random_problem(dims, N, seed=7)
    Xd, Yd = dev(X), dev(Y)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    lf = net.loss(P, Xd, Yd)
    lg, _ = net.loss_grad(P, Xd, Yd)
    assert lf == lg
    if N <= 1000:
        assert abs(lf - O.Net(dims, acts).loss(host(P), X, Y)) <= LOSS_RTOL * abs(lf)


def test_armijo_rejections_run_forward_only(ctx, pkg, monkeypatch):
    """Trials after a rejected first trial are forward + loss only until Armijo holds (the reference's
    line_search evaluates f first and Gradient only then, full_batch_minimizer.hpp:136-146); the
    trajectory is the one every other route takes (test_speculative_line_search_is_exact)."""
    monkeypatch.setenv("LBF_SPEC_DEPTH", "3")
    dims, acts = [784, 32, 10], ["relu", "linear"]
    Xh, Yh = pkg.synth_mnist(256)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(7, "cpu")
    run = pkg.LbfgsRun(net, P, dev(Xh), dev(Yh), m=5, max_iters=40, tol=0.0)
    run.iterate(40)
    info = run.info
    h = run.hist.as_dict()
    run.close()
    assert np.any(h["ls_trials"][1:] > 1)
    assert info.n_loss_only > 0
