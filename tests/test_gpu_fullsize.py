"""Oracle parity at the benched sizes: BASELINE configs 2-4 at N = 60000 (the rows bench.py times).

At N = 60000 the kernel route differs from the small-N parity tests (test_gpu_parity.py): the dW GEMM
uses 128-row tiles (above 16384 rows), the split-K plans depend on N, and the fold of the last hidden
layer's ragged dW rows runs on the 128-row tiles. These tests compare that route with the fp64 oracle
(oracle/oracle.hpp) on the same seeded data (SURVEY.md §8(d) synthetic MNIST recipe, seed 123, CPU init
stream seed 123).

Tolerances: loss relative 1e-5, gradient ||dg||/||g|| 1e-4; trajectories: the first
10 L-BFGS iterations' losses relative 1e-3 with identical line-search trial counts and pair acceptances
(src/minimizer/lbfgs.hpp:38-100, full_batch_minimizer.hpp:126-157); S-LBFGS (s_lbfgs.hpp:165-290): one
epoch's recorded loss within 5 % and the same number of live curvature pairs, the first curvature pair
(after 20 pure SVRG steps: iterate and ||s|| within 1e-4, y.s within 5e-3); the finite-difference
HVP y (s_lbfgs.hpp:88-101): ||dy||/||y|| <= 5e-2 (fp32 cancellation in w +- eps s).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N_FULL = 60000
CFG2 = ([784, 128, 10], ["relu", "linear"])
CFG3 = ([784, 128, 64, 10], ["relu", "relu", "linear"])
CFG4 = ([784, 512, 256, 10], ["relu", "relu", "linear"])
# the reference's only deep GPU workload: tests/fashion-mnist/main_gpu_deep.cpp:14-17 (784-256-128-64-10,
# ReLU x 3, Linear; L-BFGS m = 100 and m = 10 on N = 60000, :78, :92; CUDA route and init)
DEEP = ([784, 256, 128, 64, 10], ["relu", "relu", "relu", "linear"])


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()


def host(t):
    return t.double().cpu().numpy()


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


@pytest.fixture(scope="module")
def mnist(pkg):
    Xh, Yh = pkg.synth_mnist(N_FULL)
    return Xh, Yh, Xh.astype(np.float64), Yh.astype(np.float64), dev(Xh), dev(Yh)


def test_cfg2_loss_grad_full_size(ctx, pkg, O, mnist):
    _, _, X64, Y64, X, Y = mnist
    dims, acts = CFG2
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    loss, g = net.loss_grad(P, X, Y)
    l_ref, g_ref = O.Net(dims, acts).loss_grad(host(P), X64, Y64)
    assert abs(loss - l_ref) <= 1e-5 * abs(l_ref), (loss, l_ref)
    assert rel(host(g), g_ref) <= 1e-4


@pytest.mark.parametrize("dims,acts,m", [(*CFG2, 10), (*CFG3, 20), (*DEEP, 10)], ids=["cfg2_m10", "cfg3_m20", "deep_m10"])
def test_wolfe_first10_full_size(ctx, pkg, O, mnist, dims, acts, m):
    """The headline trajectory: 10 L-BFGS iterations (CPU semantics) over all 60000 rows."""
    _, _, X64, Y64, X, Y = mnist
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    P0 = host(P)
    hist, info = pkg.lbfgs_solve(net, P, X, Y, m=m, max_iters=10, tol=0.0)
    _, rec, _ = O.Net(dims, acts).lbfgs_wolfe(P0, X64, Y64, m=m, max_iters=10)
    assert len(hist["loss"]) == 10 and len(rec) == 10
    r = np.abs(hist["loss"] - rec[:, 0]) / np.abs(rec[:, 0])
    assert r.max() <= 1e-3, r
    assert np.array_equal(hist["ls_trials"], rec[:, 4].astype(int)), (hist["ls_trials"], rec[:, 4])
    assert np.array_equal(hist["accepted"][:9], rec[:9, 3].astype(int))
    g = np.abs(hist["grad_norm"][:5] - rec[:5, 1]) / np.abs(rec[:5, 1])
    assert g.max() <= 1e-3, g


@pytest.mark.parametrize("init", ["cpu", "cuda"])
def test_deep_loss_grad_full_size(ctx, pkg, O, mnist, init):
    """784-256-128-64-10 at N = 60000: three hidden layers, a 256-wide first layer (two 128-wide column tiles
    in the forward GEMM, no fused head on layer 0) and the fold on the 128 -> 64 layer's dW; both init streams
    (network.hpp:45-71 and the zero-bias network.cuh:36-59 the reference's GPU drivers use)."""
    _, _, X64, Y64, X, Y = mnist
    dims, acts = DEEP
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, init)
    loss, g = net.loss_grad(P, X, Y)
    l_ref, g_ref = O.Net(dims, acts).loss_grad(host(P), X64, Y64)
    assert abs(loss - l_ref) <= 1e-5 * abs(l_ref), (loss, l_ref)
    assert rel(host(g), g_ref) <= 1e-4


@pytest.mark.parametrize("m", [10, 100])
def test_deep_armijo_first10_full_size(ctx, pkg, O, mnist, m):
    """The deep config as the reference's GPU driver runs it (CudaLBFGS::solve, lbfgs.cuh:39-194: Armijo
    backtracking with quadratic interpolation, fp32 host scalars; CUDA init stream), 10 iterations over all
    60000 rows against the oracle's fp32 Armijo restatement: the same trial counts, losses within 1e-3."""
    Xh, Yh, _, _, X, Y = mnist
    dims, acts = DEEP
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cuda")
    P0 = host(P)
    hist, _ = pkg.lbfgs_solve(net, P, X, Y, line_search="armijo", m=m, max_iters=10, tol=0.0)
    _, rec = O.Net(dims, acts).lbfgs_armijo(P0, Xh.astype(np.float64), Yh.astype(np.float64), m=m, max_iters=10,
                                            fp32=True)
    assert len(hist["loss"]) == 10 and len(rec) == 10
    r = np.abs(hist["loss"] - rec[:, 0]) / np.abs(rec[:, 0])
    assert r.max() <= 1e-3, r
    assert np.array_equal(hist["ls_trials"], rec[:, 4].astype(int)), (hist["ls_trials"], rec[:, 4])


@pytest.mark.parametrize("N,gather", [(20000, False), (40000, False), (40000, True)])
def test_fold_128row_dw_tiles_matches_oracle(ctx, pkg, O, mnist, N, gather):
    """784-128-10 above 16384 rows: 128-row dW tiles, 784 = 6 x 128 + 16 folded columns + the bias row
    accumulated in the forward GEMM's epilogue; checked against the oracle, not only the unfolded route."""
    Xh, Yh, X64, Y64, X, Y = mnist
    dims, acts = CFG2
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(5, "cpu")
    idx = None
    rows = np.arange(N)
    if gather:
        rows = np.random.default_rng(9).permutation(N_FULL)[:N]
        idx = torch.from_numpy(rows.astype(np.int32)).cuda()
        loss, g = net.loss_grad(P, X, Y, idx=idx, l2=1e-4)
        l_ref, g_ref = O.Net(dims, acts).loss_grad(host(P), X64, Y64, idx=rows, lam=1e-4)
    else:
        loss, g = net.loss_grad(P, X[:N], Y[:N], l2=1e-4)
        l_ref, g_ref = O.Net(dims, acts).loss_grad(host(P), X64[:N], Y64[:N], lam=1e-4)
    assert abs(loss - l_ref) <= 1e-5 * abs(l_ref)
    assert rel(host(g), g_ref) <= 1e-4


@pytest.mark.parametrize("N", [16416, 30000, N_FULL])
def test_cfg3_loss_grad_full_size(ctx, pkg, O, mnist, N):
    """784-128-64-10: the middle layer's [dW ; db] keeps 128 rows in its GEMM (its bias row is folded into
    the head's epilogue) and, past 128 split-K slabs, is finished by side blocks of layer 0's dW launch:
    those must read the slabs with the folded segment size (round-2 fix; wrong before at N > ~16k)."""
    _, _, X64, Y64, X, Y = mnist
    dims, acts = CFG3
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    loss, g = net.loss_grad(P, X[:N], Y[:N])
    l_ref, g_ref = O.Net(dims, acts).loss_grad(host(P), X64[:N], Y64[:N])
    assert abs(loss - l_ref) <= 1e-5 * abs(l_ref)
    assert rel(host(g), g_ref) <= 1e-4


CFG4_KW = dict(M=10, L=10, b=256, b_H=128, step=0.005)
N_EVENTS = 24  # curvature events of one cfg-4 epoch: t = 10, 20, ..., 230 (23), one spare row


@pytest.fixture(scope="module")
def cfg4_epoch(ctx, pkg, O, mnist):
    """One full S-LBFGS epoch of cfg 4 at N = 60000 on the device (pair trace and first-pair snapshot on)
    and in the oracle's fp64 and fp32 instantiations (same host RNG stream, same records)."""
    _, _, X64, Y64, X, Y = mnist
    dims, acts = CFG4
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    P0 = host(P)
    run = pkg.SlbfgsRun(net, P, X, Y, pair_trace=64, tol=0.0, lam=1e-4, **CFG4_KW)
    pio = run.pair_io(N_EVENTS)  # record only: the run is bitwise the plain solve (checked below)
    info = run.iterate(1)
    hist, pairs = run.hist.as_dict(), run.pairs().copy()
    p0 = [host(t) for t in run.pair0()]
    pio = pio[:, :, :P0.size].cpu().numpy()
    run.close()
    onet = O.Net(dims, acts)
    okw = dict(epochs=1, tol=0.0, M=10, L=10, b=256, bH=128, step=0.005, lam=1e-4, pair_trace=64)
    o64, o32 = np.zeros(4 * P0.size), np.zeros(4 * P0.size)
    _, rec, idx64, pairs64 = onet.slbfgs(P0, X64, Y64, pair0=o64, want_idx=True, **okw)
    _, rec32, _, pairs32 = onet.slbfgs(P0, X64, Y64, fp32=True, pair0=o32, **okw)
    return dict(net=net, P0=P0, P=P, hist=hist, info=info, pairs=pairs, p0=p0, rec=rec, rec32=rec32,
                pairs64=pairs64, pairs32=pairs32, o64=o64.reshape(4, -1), o32=o32.reshape(4, -1),
                l0=float(onet.loss(P0, X64, Y64)), onet=onet, idx64=idx64, pio=pio)


def test_cfg4_slbfgs_first_pair_full_size(mnist, cfg4_epoch):
    """The first curvature pair of the cfg-4 epoch at N = 60000. The first 20 inner steps are pure SVRG (no
    pair exists until t % L == 0 with two iterate averages, s_lbfgs.hpp:218-261), then u = mean(w_10..w_20),
    s = u - u_prev and the finite-difference y on the first Hessian batch (s_lbfgs.hpp:88-101, 236-256).

    Against the fp64 oracle on the same RNG stream: the iterate w_t after the 20 steps and u within
    ||d||/||ref|| <= 1e-4; ||s|| (pair_trace row 0's s.s) within 1e-4; s itself, a difference of two averages
    10 steps apart (||s|| ~ 1e-3 ||u||, so the iterates' rounding-level differences are ~1e-3 of it), within
    1e-2. The finite difference cancels: u +- 1e-4 s moves a typical parameter by a few fp32 ulps, and a
    ReLU pre-activation within ~1e-6 of zero on one of the 128 Hessian rows changes sign between the two
    points or not depending on how they round (the step-0.01 NaN): y against the fp64 oracle's
    y (fp64 points) is a knife edge, not a tolerance (round 5: 1.2e-2 on one kernel build, a 4.6e3 vs 0.47
    y.y kink spike on the next, with w_t and s closer to fp64 on the second). Even at the device's OWN fp32
    points fl32(u +- eps s) the fp64 oracle's differenced gradients sit 5e-3 .. 7e-3 from the device's y on
    successive builds (a pre-activation within fp32 rounding of zero is on either side of the kink in fp32
    and fp64 arithmetic). So y is checked in its two non-chaotic parts: (a) the device's batch gradient at
    each of the two points against the fp64 oracle at the same points, 1e-4 as every full-size gradient test;
    (b) the device's y equal to its own two gradients differenced and scaled in fp32 (the pair sweep's
    arithmetic), and y.s (pair_trace row 0) to their y.s. The fp64-at-the-device's-points deviation and the
    fp64 oracle's own y.s are printed, with a 5e-2 sanity bound on the former."""
    _, _, X64, Y64, X, Y = mnist
    r = cfg4_epoch
    dev, o64, o32 = r["p0"], r["o64"], r["o32"]
    names = ["w_t", "u", "s", "y"]
    errs = {k: rel(dev[i], o64[i]) for i, k in enumerate(names)}
    errs32 = {k: rel(o32[i], o64[i]) for i, k in enumerate(names)}
    step = rel(dev[0] - r["P0"], o64[0] - r["P0"])  # the 20 steps' displacement alone
    row, row64, row32 = r["pairs"][0], r["pairs64"][0], r["pairs32"][0]
    # the device's FD at its own fp32 points (lincomb: fl32(u + eps s) from fp64 arithmetic), fp64 gradients
    eps = 1e-4
    u, s = dev[1], dev[2]
    wp = (u + eps * s).astype(np.float32).astype(np.float64)
    wm = (u - eps * s).astype(np.float32).astype(np.float64)
    hb = r["idx64"][21 * 256: 21 * 256 + 128]        # minibatches 0..20, then the first Hessian batch
    _, gp = r["onet"].loss_grad(wp, X64, Y64, idx=hb, lam=1e-4)
    _, gm = r["onet"].loss_grad(wm, X64, Y64, idx=hb, lam=1e-4)
    y_pts = (gp - gm) * float(np.float32(1.0 / (2.0 * eps)))
    e_pts = rel(dev[3], y_pts)
    ns, ns64 = float(np.sqrt(row[3])), float(np.sqrt(row64[3]))
    print("first pair (t = %d): " % int(row[1]) + ", ".join(f"{k} {errs[k]:.2e} (oracle fp32 {errs32[k]:.2e})"
                                                         for k in names) + f", w_t - w_0 {step:.2e}")
    print(f"first pair y.s device {row[2]:.9e} fp64 {row64[2]:.9e} fp32 {row32[2]:.9e}; ||s|| device {ns:.9e} "
          f"fp64 {ns64:.9e}; y.y device {row[4]:.9e} fp64 {row64[4]:.9e}; device y vs fp64 at its fp32 points "
          f"{e_pts:.2e}")
    # the device's own batch gradients at the two points (same 128-row batch, 1/b_H scale and lambda as the
    # solver's FD evaluations: the same plan, so the same launches)
    hbd = torch.from_numpy(hb.astype(np.int32)).cuda()
    gd = []
    for w in (wp, wm):
        Pw = torch.from_numpy(w.astype(np.float32)).cuda()
        gd.append(r["net"].loss_grad(Pw, X, Y, idx=hbd, inv_scale=1.0 / 128, l2=1e-4)[1].cpu().numpy())
    eg = [rel(gd[0].astype(np.float64), gp), rel(gd[1].astype(np.float64), gm)]
    y_own = (gd[0] - gd[1]) * np.float32(1.0 / (2.0 * eps))
    e_own = rel(dev[3], y_own.astype(np.float64))
    ys_own = float(np.dot(y_own.astype(np.float64), s))
    print(f"first pair: device batch gradients at u +- eps s vs fp64 {eg[0]:.2e} / {eg[1]:.2e}; device y vs its "
          f"own gradients differenced {e_own:.2e}; y.s {row[2]:.9e} vs {ys_own:.9e}")
    assert int(row[0]) == int(row64[0]) == 0 and int(row[1]) == int(row64[1]) == 20
    for k in ("w_t", "u"):
        assert errs[k] <= 1e-4, (k, errs[k])
    assert abs(ns - ns64) <= 1e-4 * ns64, (ns, ns64)
    assert errs["s"] <= 1e-2, errs["s"]
    assert max(eg) <= 1e-4, eg
    assert e_own <= 1e-6, e_own
    assert abs(row[2] - ys_own) <= 1e-5 * abs(ys_own), (row[2], ys_own)
    assert e_pts <= 5e-2, e_pts


def test_cfg4_slbfgs_one_epoch_full_size(ctx, pkg, O, mnist, cfg4_epoch):
    """One full S-LBFGS epoch at the cfg-4 network and N = 60000: 234 inner steps of b = 256, a curvature
    pair every L = 10 steps from the second average on (22 FD-HVPs on b_H = 128), the anchor reset and
    the recorder's full loss, all on the same host RNG stream as the oracle: the recorded loss within 5 % of
    the fp64 oracle, the same number of live pairs, bitwise reproducible (also with the pair trace off).

    Step 0.005: at cfg 4's 0.02 the synthetic problem diverges to NaN within the first epoch in the fp64
    oracle itself. Past the first pairs the epoch is sensitive at the rounding level (finite-difference
    pairs across ReLU kinks), so the per-candidate record (y.s, s.s, y.y of all 22 pairs for
    the device and both oracle instantiations) is printed beside the bound; the non-chaotic window is
    test_cfg4_slbfgs_first_pair_full_size, the step-exact parity test_gpu_parity.py::test_slbfgs_matches_oracle."""
    _, _, X64, Y64, X, Y = mnist
    r = cfg4_epoch
    hist, rec, rec32 = r["hist"], r["rec"], r["rec32"]
    P2 = r["net"].init_params(123, "cpu")
    hist2, _ = pkg.slbfgs_solve(r["net"], P2, X, Y, max_epochs=1, tol=0.0, lam=1e-4, **CFG4_KW)
    assert np.array_equal(hist["loss"], hist2["loss"]) and torch.equal(r["P"], P2)
    assert len(hist["loss"]) == 1 and len(rec) == 1 and len(rec32) == 1
    dv, o, o32 = r["pairs"], r["pairs64"], r["pairs32"]
    print("cand  t    y.s device / fp64 / fp32                    s.s device / fp64          live d/64/32")
    for i in range(min(len(dv), len(o), len(o32))):
        print(f"{i:3d} {int(dv[i, 1]):4d}  {dv[i, 2]: .6e} {o[i, 2]: .6e} {o32[i, 2]: .6e}  "
              f"{dv[i, 3]:.6e} {o[i, 3]:.6e}  {int(dv[i, 6])}/{int(o[i, 6])}/{int(o32[i, 6])}")
    dev_r = abs(hist["loss"][0] - rec[0, 0]) / abs(rec[0, 0])
    r32 = abs(rec32[0, 0] - rec[0, 0]) / abs(rec[0, 0])
    print(f"cfg4 epoch loss: device {hist['loss'][0]:.6f} oracle fp64 {rec[0, 0]:.6f} fp32 {rec32[0, 0]:.6f}: "
          f"device {dev_r:.4f}, oracle fp32 {r32:.4f} from the fp64 oracle")
    assert np.isfinite(hist["loss"][0]) and hist["loss"][0] < 0.5 * r["l0"]
    assert dev_r <= 5e-2, dev_r
    assert int(hist["accepted"][0]) == int(rec[0, 3]) == 10   # M = 10 live pairs after 22 candidates
    assert len(dv) == len(o) == 22
    assert r["info"].n_evals >= 2 * 234


def test_cfg4_tanh_slbfgs_epoch_full_size(ctx, pkg, O, mnist):
    """The cfg-4 S-LBFGS epoch on the same shape with tanh hidden layers (784-512-256-10; the reference's
    activations include tanh, src/layer.hpp): no kinks, so the finite-difference pairs are smooth functions of
    the iterates and the 234-step chain is not a knife edge; the same kernels, split-K plans and solver run
    (the activation is an epilogue parameter). Against the fp64 oracle: the epoch loss within a fixed 2 % (the
    ReLU epoch's bound is 5 %), the same live-pair count, and the 22 curvature candidates' y.s and ||s||
    printed beside the oracle's. Without kinks the pairs still part gradually (the FD's fp32 cancellation,
    test_cfg4_slbfgs_first_pair_full_size, compounds over the epoch: round 5 measured the epoch loss 6.1e-3
    from fp64, y.s up to 45 % and ||s|| up to 12 % apart at the late candidates), so the bound is fixed, not
    calibrated on any run's own spread."""
    _, _, X64, Y64, X, Y = mnist
    dims, acts = [784, 512, 256, 10], ["tanh", "tanh", "linear"]
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    P0 = host(P)
    hist, _ = pkg.slbfgs_solve(net, P, X, Y, max_epochs=1, tol=0.0, lam=1e-4, pair_trace=64, **CFG4_KW)
    onet = O.Net(dims, acts)
    _, rec, _, pairs64 = onet.slbfgs(P0, X64, Y64, epochs=1, tol=0.0, M=10, L=10, b=256, bH=128, step=0.005,
                                     lam=1e-4, pair_trace=64)
    dv = hist["pairs"]
    r = abs(hist["loss"][0] - rec[0, 0]) / abs(rec[0, 0])
    eys = np.abs(dv[:, 2] - pairs64[:, 2]) / np.abs(pairs64[:, 2])
    ess = np.abs(np.sqrt(dv[:, 3]) - np.sqrt(pairs64[:, 3])) / np.sqrt(pairs64[:, 3])
    print(f"cfg4 tanh epoch loss: device {hist['loss'][0]:.8f} oracle fp64 {rec[0, 0]:.8f}: {r:.2e}; "
          f"pairs: y.s max rel {eys.max():.2e}, ||s|| max rel {ess.max():.2e}")
    for i in range(len(dv)):
        print(f"  cand {i:2d} t {int(dv[i, 1]):3d}: y.s {dv[i, 2]: .6e} / {pairs64[i, 2]: .6e}  ||s|| "
              f"{np.sqrt(dv[i, 3]):.6e} / {np.sqrt(pairs64[i, 3]):.6e}")
    assert len(dv) == len(pairs64) == 22
    assert r <= 2e-2, r
    assert int(hist["accepted"][0]) == int(rec[0, 3])
    assert eys[0] <= 5e-2 and ess[0] <= 1e-3, (eys[0], ess[0])  # the first pair: before the FD errors compound


def test_fd_hvp_matches_oracle_cfg4(ctx, pkg, O, mnist):
    """finite_difference_hvp_batch (s_lbfgs.hpp:88-101) at the cfg-4 shape on a b_H = 128 batch: the
    device y (two fused batch evaluations at u +- 1e-4 s, fp32) vs the oracle's fp64 y. s has the scale of
    an S-LBFGS pair (L = 10 steps of 0.02 along the gradient)."""
    _, _, X64, Y64, X, Y = mnist
    dims, acts = CFG4
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    _, g = net.loss_grad(P, X, Y, l2=1e-4)
    s = (-0.2 * g).contiguous()
    rows = O.sample_indices(N_FULL, 128, seed=123, calls=1)[0]
    idx = torch.from_numpy(rows.astype(np.int32)).cuda()
    y = net.fd_hvp(P, s, X, Y, idx=idx, inv_scale=1.0 / 128, l2=1e-4, eps=1e-4)
    onet = O.Net(dims, acts)
    y_ref = onet.fd_hvp(host(P), host(s), X64, Y64, idx=rows, lam=1e-4, eps=1e-4)
    err = rel(host(y), y_ref)
    print(f"fd_hvp ||dy||/||y|| = {err:.3e}")
    assert err <= 5e-2, err
    # (the exact R-operator product is NOT a reference here: with ReLU, u +- eps s crosses kinks, and the
    # oracle's own fp64 quotient differs from H(u) s by ~30 % on this batch)
    # the device FD y is what the S-LBFGS pair sweep stores: y.s > 0 along a descent pair
    assert float((y.double() * s.double()).sum()) > 0


def test_cfg4_slbfgs_epoch_forced_pairs_full_size(ctx, pkg, O, mnist, cfg4_epoch):
    """The whole cfg-4 ReLU epoch against the fp64 oracle in a form rounding-level chaos cannot absorb (VERDICT r05
    item 1). The epoch is chaotic only through its curvature pairs: y = (g(u + eps s) - g(u - eps s)) / (2 eps)
    amplifies a rounding-level move of u across a ReLU kink by 1/(2 eps), and the ring passes that
    on to every later direction. Teacher forcing (lbf_slbfgs_pair_io, oracle PairIO) takes that channel away: the
    fp64 oracle runs the epoch with the device's u and the device's two FD gradients at each of the 23 curvature
    events, so its ring holds the device's pairs while its iterates stay its own (s_lbfgs.hpp:218-262 unchanged).
    Checked, all at fixed bounds:
      (a) every pair's two batch gradients against the fp64 oracle AT THE SAME POINTS fl32(u +- eps s) on the same
          128-row Hessian batch: 1e-4, as every full-size gradient test (22 pairs, not only the first);
      (b) the device's iterate w_{t+1} at every event against the forced oracle's: 1e-4 (the SVRG chain itself,
          234 steps of fp32 against fp64 under the same history);
      (c) the recorded epoch loss at the picked anchor against the forced oracle's: 1e-4;
      (d) the same live-pair count (the pairs' acceptance |y.s| > 1e-10, s_lbfgs.hpp:245-256, on fp32 vs fp64).
    The unforced epoch (5 % bound, test_cfg4_slbfgs_one_epoch_full_size) stays beside it."""
    _, _, X64, Y64, X, Y = mnist
    r = cfg4_epoch
    D = r["pio"].astype(np.float64)
    ne = 23
    assert not D[ne:].any() and D[:ne, 0].any()  # 23 events recorded, the spare row untouched
    assert not D[0, 2:].any() and all(D[e, 2].any() for e in range(1, ne))  # the first event offers no pair
    Ro = np.zeros_like(D)
    _, rec_f, _ = r["onet"].slbfgs(r["P0"], X64, Y64, epochs=1, tol=0.0, M=10, L=10, b=256, bH=128, step=0.005,
                                   lam=1e-4, pio_rec=Ro, pio_force=np.ascontiguousarray(D))
    eps = 1e-4
    f32 = lambda a: a.astype(np.float32).astype(np.float64)  # noqa: E731
    eg, ew = [], []
    for e in range(1, ne):
        t = 10 * (e + 1)
        u, up = D[e, 1], D[e - 1, 1]
        s = f32(u - up)
        hb = r["idx64"][256 * (t + 1) + 128 * (e - 1): 256 * (t + 1) + 128 * e]
        _, gp = r["onet"].loss_grad(f32(u + eps * s), X64, Y64, idx=hb, lam=1e-4)
        _, gm = r["onet"].loss_grad(f32(u - eps * s), X64, Y64, idx=hb, lam=1e-4)
        eg.append(max(rel(D[e, 2], gp), rel(D[e, 3], gm)))
    ew = [rel(D[e, 0], Ro[e, 0]) for e in range(ne)]
    dl = abs(r["hist"]["loss"][0] - rec_f[0, 0]) / abs(rec_f[0, 0])
    print("forced cfg-4 epoch: pair gradients at the same points vs fp64 max %.2e (per pair: %s)"
          % (max(eg), " ".join(f"{x:.1e}" for x in eg)))
    print("forced cfg-4 epoch: iterate w_t+1 vs the forced fp64 oracle max %.2e (per event: %s)"
          % (max(ew), " ".join(f"{x:.1e}" for x in ew)))
    print(f"forced cfg-4 epoch loss: device {r['hist']['loss'][0]:.9f} forced fp64 oracle {rec_f[0, 0]:.9f}: {dl:.2e}; "
          f"unforced fp64 oracle {r['rec'][0, 0]:.9f}")
    assert max(eg) <= 1e-4, eg
    assert max(ew) <= 1e-4, ew
    assert dl <= 1e-4, dl
    assert int(r["hist"]["accepted"][0]) == int(rec_f[0, 3])


@pytest.mark.parametrize("dims,acts,init,line_search", [(*CFG2, "cpu", "wolfe"), (*CFG2, "cpu", "armijo"),
                                                      (*CFG3, "cpu", "wolfe"), (*DEEP, "cuda", "armijo")],
                         ids=["cfg2_wolfe", "cfg2_armijo", "cfg3_wolfe", "deep_armijo"])
def test_early_armijo_exit_bitwise(ctx, pkg, mnist, monkeypatch, dims, acts, init, line_search):
    """EarlyLs (csrc/kernels.hpp, gemm.hip gemm_early_exit): a speculative first trial that fails sufficient
    decrease (full_batch_minimizer.hpp:138-141 / lbfgs.cuh:159-163) is rejected by its first backward GEMM, which
    skips the trial's backward and tail. Over 60 iterations at N = 60000 (cfg 2, and cfg 3 and the deep net,
    whose first backward launch is a hidden layer's dW GEMM with the fold) the trajectory and the final parameters are bitwise those with the test
    left to the fused tail (LBF_NO_EARLY=1), and each skipped backward is one full evaluation fewer and one
    loss-only trial more."""
    _, _, _, _, X, Y = mnist
    net = pkg.Mlp(ctx, dims, acts)
    runs = {}
    for off in (True, False):
        if off:
            monkeypatch.setenv("LBF_NO_EARLY", "1")
        else:
            monkeypatch.delenv("LBF_NO_EARLY", raising=False)
        P = net.init_params(123, init)
        hist, info = pkg.lbfgs_solve(net, P, X, Y, m=10, max_iters=60, tol=0.0, line_search=line_search)
        runs[off] = (hist, int(info.n_evals), int(info.n_loss_only), host(P))
    (h0, e0, l0, p0), (h1, e1, l1, p1) = runs[True], runs[False]
    for k in ("loss", "grad_norm", "alpha", "ls_trials", "accepted"):
        assert np.array_equal(h0[k], h1[k]), k
    assert np.array_equal(p0, p1)
    skipped = l1 - l0
    print(f"{dims} {line_search}: {skipped} first trials rejected early in 60 iterations ({e0} -> {e1} full evaluations)")
    assert e0 - e1 == skipped >= 0
    if dims == CFG2[0] and line_search == "wolfe":
        assert skipped > 0  # cfg 2 rejects ~5 % of its first trials on sufficient decrease
