"""The product's multi-rank path (nranks > 1) on ONE GPU, through an in-process rank group.

RCCL refuses two ranks on one device, so `lbf_comm_init_local` (csrc/comm.cpp) makes 2-4 contexts on
GPU 0 the ranks of one group: each rank is driven by its own host thread (as one process per GPU would
drive it), evaluates its contiguous shard / minibatch slice, and the group's all-reduce sums every
rank's [grad | sse_hi | sse_lo] buffer on the device in rank order. Everything the driver's 8-GPU run
executes with nranks > 1 runs here: rank > 0 shard offsets, the n_global scaling, the S-LBFGS slices
b*rk/nr .. b*(rk+1)/nr of every minibatch, Hessian batch and anchor, empty shares (b < world), the
(hi, lo) loss words of different shards summed, and line-search decisions replicated on summed data.

The reference has no collective; the split rests on the loss being a sum over samples
(src/unified_optimization.hpp:101-120, src/cuda/network.cuh:105-107) and on S-LBFGS's batch_g
(unified_optimization.hpp:343-400, s_lbfgs.hpp:218-262). Tolerances ("1-GPU vs 8-GPU:
per-call rel <= 1e-5"): the shard sums are added in another order than one GPU's split-K slabs, so
results agree to fp32 rounding, not bitwise; ranks of one group agree bitwise with each other.
"""
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()


def host(t):
    return t.double().cpu().numpy()


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def run_ranks(pkg, world, body, timeout=240):
    """body(rank, ctx) on `world` threads, each rank of one in-process group on GPU 0."""
    ctxs = [pkg.Context(0, use_torch_stream=False) for _ in range(world)]
    pkg.Context.comm_init_local(ctxs)
    torch.cuda.synchronize()
    out, err = [None] * world, [None] * world

    def th(r):
        try:
            torch.cuda.set_device(0)
            out[r] = body(r, ctxs[r])
            torch.cuda.synchronize()
        except BaseException as e:  # noqa: BLE001 (re-raised below)
            err[r] = e

    ts = [threading.Thread(target=th, args=(r,), daemon=True) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout)
    assert not any(t.is_alive() for t in ts), "a rank thread did not finish"
    for e in err:
        if e is not None:
            raise e
    return out


def shard(N, world, r):
    return N * r // world, N * (r + 1) // world


def test_local_group_allreduce(pkg):
    """Rank-order device sum, identical on every rank; counts up to 16 ranks' worth of data."""
    world = 3
    base = [torch.randn(100003, device="cuda") for _ in range(world)]
    bufs = [b.clone() for b in base]

    def body(r, c):
        c.allreduce_(bufs[r])
        c.allreduce_(bufs[r])  # twice: the group's events and barrier are reused
        return None

    run_ranks(pkg, world, body)
    s1 = (base[0] + base[1]) + base[2]
    s2 = (s1 + s1) + s1
    for r in range(world):
        assert torch.equal(bufs[r], s2)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("dims,acts,N", [([784, 128, 10], ["relu", "linear"], 7501),
                                         ([784, 128, 64, 10], ["relu", "relu", "linear"], 3000),
                                         ([784, 300, 20], ["tanh", "linear"], 1001)])
def test_ranks_loss_grad_equals_single(ctx, pkg, world, dims, acts, N):
    Xh, Yh = pkg.synth_mnist(N, dims[0], dims[-1])
    net1 = pkg.Mlp(ctx, dims, acts)
    P = net1.init_params(123, "cpu")
    l1, g1 = net1.loss_grad(P, dev(Xh), dev(Yh), inv_scale=1.0 / N)
    shards = [shard(N, world, r) for r in range(world)]
    Xs = [dev(Xh[lo:hi]) for lo, hi in shards]
    Ys = [dev(Yh[lo:hi]) for lo, hi in shards]

    def body(r, c):
        net = pkg.Mlp(c, dims, acts)
        return net.loss_grad(P, Xs[r], Ys[r], inv_scale=1.0 / N)

    res = run_ranks(pkg, world, body)
    for lr, gr in res:
        assert lr == res[0][0] and torch.equal(gr, res[0][1])  # replicated, bitwise
    assert abs(res[0][0] - l1) <= 1e-6 * abs(l1)
    assert rel(host(res[0][1]), host(g1)) <= 1e-5


def test_ranks_minibatch_slices_equal_single(ctx, pkg):
    """S-LBFGS batch_g on a sampled minibatch: each rank evaluates its slice of the index list with the
    whole batch's 1/b scale and lambda; the group sum equals the single evaluation of the whole list."""
    dims, acts = [784, 512, 256, 10], ["relu", "relu", "linear"]
    N, b, world = 60000, 256, 2
    Xh, Yh = pkg.synth_mnist(N)
    X, Y = dev(Xh), dev(Yh)
    idx = torch.from_numpy(pkg.sample_indices(N, b, 123)[0].astype(np.int32)).cuda()
    net1 = pkg.Mlp(ctx, dims, acts)
    P = net1.init_params(123, "cpu")
    l1, g1 = net1.loss_grad(P, X, Y, idx=idx, inv_scale=1.0 / b, l2=1e-4)

    def body(r, c):
        lo, hi = shard(b, world, r)
        net = pkg.Mlp(c, dims, acts)
        return net.loss_grad(P, X, Y, idx=idx[lo:hi].contiguous(), inv_scale=1.0 / b, l2=1e-4)

    res = run_ranks(pkg, world, body)
    assert torch.equal(res[0][1], res[1][1])
    assert abs(res[0][0] - l1) <= 1e-6 * abs(l1)
    assert rel(host(res[0][1]), host(g1)) <= 1e-5


@pytest.mark.parametrize("line_search", ["wolfe", "armijo"])
def test_ranks_cfg2_full_size_trajectory(ctx, pkg, line_search):
    """BASELINE cfg 2 at N = 60000 split 30000 / 30000: 10 L-BFGS iterations with the same line-search
    trial counts and pair acceptances as the single route, losses within 1e-5, ranks bitwise identical."""
    dims, acts, N, world = [784, 128, 10], ["relu", "linear"], 60000, 2
    Xh, Yh = pkg.synth_mnist(N)
    net1 = pkg.Mlp(ctx, dims, acts)
    P0 = net1.init_params(123, "cpu")
    P1 = P0.clone()
    h1, _ = pkg.lbfgs_solve(net1, P1, dev(Xh), dev(Yh), line_search=line_search, m=10, max_iters=10, tol=0.0)
    shards = [shard(N, world, r) for r in range(world)]
    Xs = [dev(Xh[lo:hi]) for lo, hi in shards]
    Ys = [dev(Yh[lo:hi]) for lo, hi in shards]

    def body(r, c):
        net = pkg.Mlp(c, dims, acts)
        P = P0.clone()
        h, info = pkg.lbfgs_solve(net, P, Xs[r], Ys[r], n_global=N, line_search=line_search, m=10, max_iters=10,
                                  tol=0.0)
        return h, P, info.n_rows

    res = run_ranks(pkg, world, body)
    for h, P, _ in res[1:]:
        assert np.array_equal(h["loss"], res[0][0]["loss"]) and torch.equal(P, res[0][1])
    assert res[0][2] == res[1][2] > 0  # 30000 rows per evaluation on each rank
    h = res[0][0]
    assert np.array_equal(h["ls_trials"], h1["ls_trials"]), (h["ls_trials"], h1["ls_trials"])
    assert np.array_equal(h["accepted"], h1["accepted"])
    assert np.max(np.abs(h["loss"] - h1["loss"]) / np.abs(h1["loss"])) <= 1e-5
    assert rel(host(res[0][1]), host(P1)) <= 1e-4


@pytest.mark.parametrize("world", [3, 4])
def test_ranks_ragged_lbfgs(ctx, pkg, world):
    """Ragged shards (N = 2049 over 3 / 4 ranks), Wolfe and the speculative pipeline with rejections:
    ranks bitwise identical, the first 10 iterations as the single route's."""
    dims, acts, N = [784, 64, 10], ["relu", "linear"], 2049
    Xh, Yh = pkg.synth_mnist(N)
    net1 = pkg.Mlp(ctx, dims, acts)
    P0 = net1.init_params(7, "cpu")
    P1 = P0.clone()
    h1, _ = pkg.lbfgs_solve(net1, P1, dev(Xh), dev(Yh), m=10, max_iters=25, tol=0.0)
    shards = [shard(N, world, r) for r in range(world)]
    Xs = [dev(Xh[lo:hi]) for lo, hi in shards]
    Ys = [dev(Yh[lo:hi]) for lo, hi in shards]

    def body(r, c):
        net = pkg.Mlp(c, dims, acts)
        P = P0.clone()
        h, _ = pkg.lbfgs_solve(net, P, Xs[r], Ys[r], n_global=N, m=10, max_iters=25, tol=0.0)
        return h, P

    res = run_ranks(pkg, world, body)
    for h, P in res[1:]:
        assert np.array_equal(h["loss"], res[0][0]["loss"]) and torch.equal(P, res[0][1])
    h = res[0][0]
    assert np.array_equal(h["ls_trials"][:10], h1["ls_trials"][:10])
    assert np.max(np.abs(h["loss"][:10] - h1["loss"][:10]) / np.abs(h1["loss"][:10])) <= 1e-4


def test_ranks_empty_share_lbfgs(ctx, pkg):
    """N = 3 rows over 4 ranks: one rank evaluates nothing and still joins every all-reduce."""
    dims, acts, N, world = [784, 16, 10], ["relu", "linear"], 3, 4
    Xh, Yh = pkg.synth_mnist(N)
    net1 = pkg.Mlp(ctx, dims, acts)
    P0 = net1.init_params(3, "cpu")
    P1 = P0.clone()
    h1, _ = pkg.lbfgs_solve(net1, P1, dev(Xh), dev(Yh), m=5, max_iters=8, tol=0.0)
    shards = [shard(N, world, r) for r in range(world)]
    Xs = [dev(Xh[lo:hi]) if hi > lo else dev(np.zeros((1, 784))) for lo, hi in shards]
    Ys = [dev(Yh[lo:hi]) if hi > lo else dev(np.zeros((1, 10))) for lo, hi in shards]

    def body(r, c):
        net = pkg.Mlp(c, dims, acts)
        P = P0.clone()
        lo, hi = shards[r]
        h, _ = pkg.lbfgs_solve(net, P, Xs[r][: hi - lo], Ys[r][: hi - lo], n_global=N, m=5, max_iters=8, tol=0.0)
        return h, P

    res = run_ranks(pkg, world, body)
    for h, P in res[1:]:
        assert torch.equal(P, res[0][1])
    h = res[0][0]
    assert np.array_equal(h["ls_trials"], h1["ls_trials"])
    assert np.max(np.abs(h["loss"] - h1["loss"]) / np.abs(h1["loss"])) <= 1e-4


@pytest.mark.parametrize("world,kw", [
    (2, dict(M=5, L=4, b=32, b_H=16)),
    (3, dict(M=5, L=4, b=32, b_H=16)),
    # b < world: one rank's slice of every minibatch and Hessian batch is empty. The finite-difference pair of
    # a one-row Hessian batch amplifies the two routes' rounding-level differences by ~1/(2 eps) (with ReLU
    # kinks, chaotically: one epoch < 5 % apart on round 4's build, 24.6 % on round 5's re-rounded head; with
    # tanh still 2.5 %), so the empty-slice path is compared on the smooth network with the exact HVP pairs,
    # at the default fixed bound
    (2, dict(M=5, L=4, b=1, b_H=1, step=0.002, hvp_exact=1, acts=["tanh", "linear"])),
    (2, dict(M=5, L=4, b=32, b_H=1, hvp_exact=1)),  # exact HVP with b_H < world
    # replicated inner steps: identical chains on every rank, the full-batch gradient sharded
    (2, dict(M=5, L=4, b=32, b_H=16, dp_mode="replicated")),
    (3, dict(M=5, L=4, b=32, b_H=16, dp_mode="replicated")),
    (4, dict(M=5, L=4, b=32, b_H=1, hvp_exact=1, dp_mode="replicated")),
])
def test_ranks_slbfgs_equals_single(ctx, pkg, world, kw):
    kw = dict(kw)
    dims, acts, N = [784, 16, 10], kw.pop("acts", ["relu", "linear"]), 512 if kw["b"] > 1 else 64
    Xh, Yh = pkg.synth_mnist(N)
    X, Y = dev(Xh), dev(Yh)
    rtol = kw.pop("rtol", 1e-3)
    args = dict(step=0.02, max_epochs=2, tol=0.0, lam=1e-4, dp_mode="sliced")
    args.update(kw)
    net1 = pkg.Mlp(ctx, dims, acts)
    P0 = net1.init_params(123, "cpu")
    P1 = P0.clone()
    h1, _ = pkg.slbfgs_solve(net1, P1, X, Y, **args)

    def body(r, c):
        net = pkg.Mlp(c, dims, acts)
        P = P0.clone()
        h, _ = pkg.slbfgs_solve(net, P, X, Y, **args)
        return h, P

    res = run_ranks(pkg, world, body)
    for h, P in res[1:]:
        assert np.array_equal(h["loss"], res[0][0]["loss"]) and torch.equal(P, res[0][1])
    h = res[0][0]
    assert np.all(np.isfinite(h["loss"]))
    assert np.array_equal(h["accepted"], h1["accepted"])
    # two epochs of SVRG steps with FD curvature pairs: rounding-level differences grow (the small-N oracle
    # parity test of the same configuration, test_gpu_parity.py::test_slbfgs_matches_oracle, uses 1e-3)
    assert np.max(np.abs(h["loss"] - h1["loss"]) / np.abs(h1["loss"])) <= rtol, (h["loss"], h1["loss"])
    assert rel(host(res[0][1]), host(P1)) <= 10 * rtol


@pytest.mark.parametrize("moved", ["start", "never"])
def test_ranks_replicated_drift_fails_loudly(ctx, pkg, moved):
    """Replicated S-LBFGS data parallelism is only correct while every rank's inner-step chain is bitwise the
    same (nothing is exchanged inside an epoch): each full-batch evaluation first all-reduces fingerprints of
    every rank's anchor and fails on a mismatch, instead of summing shard gradients taken at different points.
    Rank 1 given parameters moved by 2 ulp must fail on every rank; identical ones must pass."""
    dims, acts, N, world = [784, 16, 10], ["relu", "linear"], 512, 2
    Xh, Yh = pkg.synth_mnist(N)
    X, Y = dev(Xh), dev(Yh)
    args = dict(M=5, L=4, b=32, b_H=16, step=0.02, max_epochs=2, tol=0.0, lam=1e-4, dp_mode="replicated")
    P0 = pkg.Mlp(ctx, dims, acts).init_params(123, "cpu")

    def body(r, c):
        net = pkg.Mlp(c, dims, acts)
        P = P0.clone()
        if r == 1 and moved == "start":
            P.mul_(1.0 + 2.0 ** -22)
        try:
            h, _ = pkg.slbfgs_solve(net, P, X, Y, **args)
        except pkg.LbfError as e:
            return str(e)
        return h

    res = run_ranks(pkg, world, body)
    if moved == "start":
        assert all(isinstance(r, str) and "drifted apart" in r for r in res), res
    else:
        assert all(isinstance(r, dict) for r in res) and np.array_equal(res[0]["loss"], res[1]["loss"])


@pytest.mark.parametrize("dp_mode", ["sliced", "replicated"])
def test_ranks_cfg4_epoch(ctx, pkg, dp_mode):
    """BASELINE cfg 4 (784-512-256-10, N = 60000, b = 256, b_H = 128, L = M = 10) for one epoch at world 2
    against the single route. Sliced: the twin's anchor gradients ahead and ONE all-reduce per [g(w_t) | g(w)]
    block. Replicated: every rank runs the whole chain, the full-batch gradient at the anchor is sharded.

    The two routes add the full-batch gradient's shard sums (and, sliced, every minibatch gradient) in
    another order, so they start apart at the rounding level; past the first finite-difference pairs the
    ReLU epoch is chaotic at that level (tests/test_gpu_fullsize.py: re-rounding the head epilogue alone moved
    the single route's epoch loss by 3.4 %, and this comparison from 0.9 % to 5.7 %). The fixed-bound checks
    are therefore the non-chaotic window and the smooth network: the iterate after the first 20 (pure SVRG)
    steps and their average u, the first pair's s (pair_trace snapshot), within 1e-4 / 1e-4 / 1e-2 of the
    single route; the same live-pair count; ranks bitwise identical; and the same epoch with tanh hidden
    layers within a fixed 2 % (test_ranks_cfg4_tanh_epoch). The ReLU epoch loss is printed beside them."""
    dims, acts, N, world = [784, 512, 256, 10], ["relu", "relu", "linear"], 60000, 2
    Xh, Yh = pkg.synth_mnist(N)
    X, Y = dev(Xh), dev(Yh)
    args = dict(M=10, L=10, b=256, b_H=128, step=0.005, tol=0.0, lam=1e-4, dp_mode=dp_mode)
    net1 = pkg.Mlp(ctx, dims, acts)
    P0 = net1.init_params(123, "cpu")
    run1 = pkg.SlbfgsRun(net1, P0.clone(), X, Y, pair_trace=64, **args)
    i1 = run1.iterate(1)
    h1, p01 = run1.hist.as_dict(), [host(t) for t in run1.pair0()]
    run1.close()

    def body(r, c):
        net = pkg.Mlp(c, dims, acts)
        P = P0.clone()
        run = pkg.SlbfgsRun(net, P, X, Y, pair_trace=64, **args)
        info = run.iterate(1)
        out = run.hist.as_dict(), [host(t) for t in run.pair0()], info.n_rows, P
        run.close()
        return out

    res = run_ranks(pkg, world, body)
    assert torch.equal(res[0][3], res[1][3])
    h, p0 = res[0][0], res[0][1]
    assert np.isfinite(h["loss"][0])
    assert h["accepted"][0] == h1["accepted"][0]
    e = [rel(p0[i], p01[i]) for i in range(3)]
    d = abs(h["loss"][0] - h1["loss"][0]) / abs(h1["loss"][0])
    print(f"cfg4 epoch, world 2 {dp_mode}: first pair w_t {e[0]:.2e} u {e[1]:.2e} s {e[2]:.2e} from the single "
          f"route; epoch loss {h['loss'][0]:.6f} single route {h1['loss'][0]:.6f}: {d:.4f}")
    assert e[0] <= 1e-4 and e[1] <= 1e-4 and e[2] <= 1e-2, e
    if dp_mode == "sliced":
        assert res[0][2] + res[1][2] == i1.n_rows  # the ranks' slices partition the single route's rows
    else:  # every rank evaluates every minibatch row; the two full-batch evaluations are split
        full = 2 * N
        assert res[0][2] + res[1][2] == 2 * (i1.n_rows - full) + full


@pytest.mark.parametrize("dp_mode", ["sliced", "replicated"])
def test_ranks_cfg4_tanh_epoch(ctx, pkg, dp_mode):
    """The cfg-4 epoch at world 2 on the smooth network (tanh hidden layers: no kinks for the finite
    differences to cross): epoch loss within a fixed 2 % of the single route, the same live-pair count."""
    dims, acts, N, world = [784, 512, 256, 10], ["tanh", "tanh", "linear"], 60000, 2
    Xh, Yh = pkg.synth_mnist(N)
    X, Y = dev(Xh), dev(Yh)
    args = dict(M=10, L=10, b=256, b_H=128, step=0.005, max_epochs=1, tol=0.0, lam=1e-4, dp_mode=dp_mode)
    net1 = pkg.Mlp(ctx, dims, acts)
    P0 = net1.init_params(123, "cpu")
    h1, _ = pkg.slbfgs_solve(net1, P0.clone(), X, Y, **args)

    def body(r, c):
        net = pkg.Mlp(c, dims, acts)
        P = P0.clone()
        h, _ = pkg.slbfgs_solve(net, P, X, Y, **args)
        return h, P

    res = run_ranks(pkg, world, body)
    assert torch.equal(res[0][1], res[1][1])
    h = res[0][0]
    d = abs(h["loss"][0] - h1["loss"][0]) / abs(h1["loss"][0])
    print(f"cfg4 tanh epoch, world 2 {dp_mode}: loss {h['loss'][0]:.8f} single route {h1['loss'][0]:.8f}: {d:.2e}")
    assert h["accepted"][0] == h1["accepted"][0]
    assert d <= 2e-2, d


def _forced_routes(ctx, pkg, dims, acts, X, Y, args, world, cap, seed=123):
    """The single route records its curvature events (lbf_slbfgs_pair_io); then the world-`world` rank group runs
    the same solve teacher-forced with that record (its ring receives the single route's pairs, its iterates and
    its FD gradients at the forced points stay its own) and records too. Returns (single, ranks) as
    (history, record [cap, 4, n] on the host, params)."""
    net1 = pkg.Mlp(ctx, dims, acts)
    P0 = net1.init_params(seed, "cpu")
    n = P0.numel()
    run1 = pkg.SlbfgsRun(net1, P0.clone(), X, Y, **args)
    rec1 = run1.pair_io(cap)
    run1.iterate(args.get("max_epochs", 1))
    single = (run1.hist.as_dict(), rec1[:, :, :n].double().cpu().numpy(), run1._keep[1].clone())
    run1.close()

    def body(r, c):
        net = pkg.Mlp(c, dims, acts)
        P = P0.clone()
        run = pkg.SlbfgsRun(net, P, X, Y, **args)
        rec = run.pair_io(cap, force=rec1)
        run.iterate(args.get("max_epochs", 1))
        out = run.hist.as_dict(), rec[:, :, :n].double().cpu().numpy(), P
        run.close()
        return out

    return single, run_ranks(pkg, world, body)


@pytest.mark.parametrize("dp_mode", ["sliced", "replicated"])
def test_ranks_cfg4_epoch_forced_pairs(ctx, pkg, dp_mode):
    """The world-2 ReLU cfg-4 epoch (784-512-256-10, N = 60000, b = 256, b_H = 128, L = M = 10) against the single
    route over the WHOLE epoch, in a form the FD pairs' kink chaos cannot absorb. The world-2
    route is teacher-forced with the single route's curvature events (u and the two FD gradients of each of the 23
    events, lbf_slbfgs_pair_io): its ring then holds the single route's 22 pairs, while each event's gradients are
    still evaluated by the world-2 route at the (forced, so identical) points u +- eps s, and its iterates are its
    own. Checked at fixed bounds:
      - each pair's two FD gradients at the same points: sliced, the ranks' Hessian-batch slices summed by the
        all-reduce, 1e-5 (the shard-sum tolerance); replicated, the pair evaluations run inside the rank-local
        chain, so bitwise;
      - the iterate w_{t+1} at every event and the own average u: 1e-4 of the single route (sliced: every
        minibatch gradient summed across ranks; replicated: only the full-batch anchor gradient is);
      - the epoch loss: 1e-4; the same live-pair count; ranks bitwise identical.
    The unforced ReLU epoch's distance stays printed in test_ranks_cfg4_epoch."""
    dims, acts, N, world = [784, 512, 256, 10], ["relu", "relu", "linear"], 60000, 2
    Xh, Yh = pkg.synth_mnist(N)
    X, Y = dev(Xh), dev(Yh)
    args = dict(M=10, L=10, b=256, b_H=128, step=0.005, tol=0.0, lam=1e-4, dp_mode=dp_mode, max_epochs=1)
    (h1, R1, _), res = _forced_routes(ctx, pkg, dims, acts, X, Y, args, world, 24)
    assert torch.equal(res[0][2], res[1][2]) and np.array_equal(res[0][1], res[1][1])
    h, R = res[0][0], res[0][1]
    ne = 23
    eg = [max(rel(R[e, 2], R1[e, 2]), rel(R[e, 3], R1[e, 3])) for e in range(1, ne)]
    ew = [rel(R[e, 0], R1[e, 0]) for e in range(ne)]
    eu = [rel(R[e, 1], R1[e, 1]) for e in range(ne)]
    dl = abs(h["loss"][0] - h1["loss"][0]) / abs(h1["loss"][0])
    print(f"forced cfg4 epoch, world 2 {dp_mode}: FD gradients at the same points max {max(eg):.2e}; iterate max "
          f"{max(ew):.2e} (last {ew[-1]:.2e}); u max {max(eu):.2e}; epoch loss {h['loss'][0]:.9f} single "
          f"{h1['loss'][0]:.9f}: {dl:.2e}")
    if dp_mode == "replicated":
        assert max(eg) == 0.0, eg
    else:
        assert max(eg) <= 1e-5, eg
    assert max(ew) <= 1e-4 and max(eu) <= 1e-4, (ew, eu)
    assert dl <= 1e-4, dl
    assert h["accepted"][0] == h1["accepted"][0]


@pytest.mark.parametrize("hvp_exact", [0, 1])
def test_ranks_fd_pairs_empty_slice_forced(ctx, pkg, hvp_exact):
    """b_H = 1 < world = 2, sliced: rank 1's slice of every Hessian batch is EMPTY, so each
    curvature pair is one rank's one-row evaluation plus an empty one, summed by the all-reduce, with lambda w added
    once after it. Teacher-forced with the single route's events, each pair's gradients (the reference's finite
    difference, hvp_exact = 0; and the exact HVP) are compared with the single route's AT THE SAME POINTS, every pair
    of two epochs: within 1e-6 (a sum with zeros in another order); the iterates under the same history within 1e-4."""
    dims, acts, N, world = [784, 16, 10], ["relu", "linear"], 512, 2
    Xh, Yh = pkg.synth_mnist(N)
    X, Y = dev(Xh), dev(Yh)
    args = dict(M=5, L=4, b=32, b_H=1, step=0.02, tol=0.0, lam=1e-4, dp_mode="sliced", max_epochs=2,
                hvp_exact=hvp_exact)
    cap = 2 * (N // 32 // 4) + 2
    (h1, R1, _), res = _forced_routes(ctx, pkg, dims, acts, X, Y, args, world, cap)
    assert torch.equal(res[0][2], res[1][2])
    h, R = res[0][0], res[0][1]
    ev = [e for e in range(cap) if R1[e, 2].any()]
    assert len(ev) == 2 * ((N // 32 - 1) // 4) - 1  # t = 4, 8, 12 per epoch; every event but the first: a pair
    eg = [max(rel(R[e, 2], R1[e, 2]), rel(R[e, 3], R1[e, 3]) if R1[e, 3].any() else 0.0) for e in ev]
    ew = [rel(R[e, 0], R1[e, 0]) for e in ev]
    print(f"b_H = 1 over 2 ranks (hvp_exact {hvp_exact}): pair gradients at the same points max {max(eg):.2e}; "
          f"iterates max {max(ew):.2e}; losses {h['loss']} single {h1['loss']}")
    assert max(eg) <= 1e-6, eg
    assert max(ew) <= 1e-4, ew
    assert np.array_equal(h["accepted"], h1["accepted"])
    assert np.max(np.abs(h["loss"] - h1["loss"]) / np.abs(h1["loss"])) <= 1e-4
