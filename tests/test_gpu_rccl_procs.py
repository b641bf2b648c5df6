"""The product's cross-process RCCL path (one process per rank, `lbf_comm_init` with a broadcast unique id)
executed on a one-GPU box (until now only a 1-rank communicator and the in-process rank
group had run it).

Both ranks run on GPU 0. RCCL refuses two ranks of one host on one device, so each rank process gets its
own NCCL_HOSTID: RCCL then treats them as two hosts and connects them through its socket transport on the
loopback interface (tests/rccl_worker.py). Everything above the wire is what the driver's N-GPU run
executes: gloo control plane, the id broadcast, communicator creation, the all-reduce inside each
data-parallel evaluation (L-BFGS shards, S-LBFGS sliced minibatches, the replicated mode's full-batch
gradient and its anchor fingerprints), and bench.py's own rank code.

Oracle for the library check: the in-process rank group at the same world size (tests/test_gpu_ranks.py,
itself checked against the single route and the CPU oracle). At world 2 an all-reduce adds two fp32
terms, which is order-independent, so RCCL and the rank group must agree BITWISE on every output.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)

import rccl_worker  # noqa: E402
from test_gpu_ranks import run_ranks  # noqa: E402

pytestmark = pytest.mark.gpu


def free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def rank_env(rank, world, port):
    e = dict(os.environ)
    e.update(RANK=str(rank), LOCAL_RANK="0", WORLD_SIZE=str(world), LOCAL_WORLD_SIZE="1", GROUP_RANK=str(rank),
             MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
             NCCL_HOSTID=f"lbf-test-rank{rank}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return e


def run_procs(cmds, timeout):
    """Start one process per rank, each writing to its own file (no pipe can fill and block a rank); poll every
    rank, and kill the others as soon as one exits non-zero (a rank left in a collective would wait for the
    dead one until the time limit) or the group overruns `timeout`."""
    import tempfile
    import time

    logs = [tempfile.TemporaryFile(mode="w+") for _ in cmds]
    procs = [subprocess.Popen(c, env=e, stdout=f, stderr=subprocess.STDOUT, text=True, cwd=ROOT)
             for (c, e), f in zip(cmds, logs)]
    t_end = time.monotonic() + timeout
    failed = None
    while any(p.poll() is None for p in procs):
        bad = [r for r, p in enumerate(procs) if p.poll() not in (None, 0)]
        if bad or time.monotonic() > t_end:
            failed = bad[0] if bad else -1
            break
        time.sleep(0.2)
    if failed is not None:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for p in procs:
            p.wait()
    outs = []
    for f in logs:
        f.seek(0)
        outs.append(f.read())
        f.close()
    if failed == -1:
        pytest.fail("a rank process overran its time limit:\n" + "\n".join(o[-2000:] for o in outs))
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{outs[r][-4000:]}"
    return outs


@pytest.fixture(scope="module")
def rccl2(tmp_path_factory):
    prefix = str(tmp_path_factory.mktemp("rccl") / "w2")
    world, port = 2, free_port()
    run_procs([([sys.executable, "-u", os.path.join(HERE, "rccl_worker.py"), prefix], rank_env(r, world, port))
               for r in range(world)], timeout=300)
    return [dict(np.load(f"{prefix}.rank{r}.npz")) for r in range(world)]


@pytest.fixture(scope="module")
def group2(pkg):
    return run_ranks(pkg, 2, lambda r, c: rccl_worker.run_rank(pkg, c, r, 2))


def test_rccl_ranks_replicated(rccl2):
    """Every output is replicated across the two processes, bit for bit."""
    a, b = rccl2
    assert a.keys() == b.keys()
    for k in a:
        if k.endswith("_rows"):
            continue
        assert np.array_equal(a[k], b[k]), k


def test_rccl_allreduce_sum(rccl2):
    x0, x1 = (rccl_worker.allreduce_input(r) for r in range(2))
    assert np.array_equal(rccl2[0]["allreduce"], (x0 + x1).numpy())


def test_rccl_equals_rank_group(rccl2, group2):
    """RCCL across processes == the in-process rank group, bitwise: cfg-2 loss/gradient at N = 60000 split
    30000 / 30000, 10 Wolfe and 10 Armijo iterations (losses, trial counts, acceptances, final parameters),
    two S-LBFGS epochs in both data-parallel modes."""
    a, g = rccl2[0], group2[0]
    for k in a:
        assert np.array_equal(a[k], g[k]), k
    assert a["wolfe_rows"] > 0


def test_rccl_against_single_route(ctx, pkg, rccl2):
    """The cross-process result against one rank evaluating all 60000 rows (fp32 rounding of another
    summation order), the single route's Wolfe trajectory with the same trials and acceptances."""
    dims, acts, N = rccl_worker.CFG2
    Xh, Yh = pkg.synth_mnist(N)
    X, Y = rccl_worker.dev(Xh), rccl_worker.dev(Yh)
    net = pkg.Mlp(ctx, dims, acts)
    P0 = net.init_params(123, "cpu")
    l1, g1 = net.loss_grad(P0, X, Y, inv_scale=1.0 / N)
    a = rccl2[0]
    assert abs(a["cfg2_loss"] - l1) <= 1e-6 * abs(l1)
    g1 = g1.double().cpu().numpy()
    assert np.linalg.norm(a["cfg2_grad"] - g1) <= 1e-5 * np.linalg.norm(g1)
    P = P0.clone()
    h1, _ = pkg.lbfgs_solve(net, P, X, Y, line_search="wolfe", m=10, max_iters=10, tol=0.0)
    assert np.array_equal(a["wolfe_trials"], h1["ls_trials"]) and np.array_equal(a["wolfe_accepted"], h1["accepted"])
    assert np.max(np.abs(a["wolfe_loss"] - h1["loss"]) / np.abs(h1["loss"])) <= 1e-5


@pytest.mark.parametrize("solver,world", [("lbfgs", 2), ("slbfgs", 2), ("lbfgs", 4)])
def test_bench_two_ranks_one_gpu(solver, world, tmp_path):
    """bench.py as the driver runs it at N = 2 and 4 (WORLD_SIZE set, one process per rank, the RCCL id through
    gloo, the barrier + max-over-ranks clock; at 4 ranks also shard offsets past the second rank), every rank
    on GPU 0: one JSON line from rank 0 with n_gpus N / dpN and a finite value. The timing of ranks sharing one
    GPU over sockets is not a result."""
    port = free_port()
    args = ["--gpus", str(world), "--steps", "3" if solver == "slbfgs" else "10", "--warmup", "1", "--no-cpu-baseline",
            "--device-warmup", "0", "--solver", solver]
    outs = run_procs([([sys.executable, "-u", os.path.join(ROOT, "bench.py")] + args, rank_env(r, world, port))
                      for r in range(world)], timeout=300)
    lines = [ln for ln in outs[0].splitlines() if ln.startswith("{")]
    assert len(lines) == 1, outs[0][-3000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["config"]["parallelism"].startswith(f"dp{world}")
    assert np.isfinite(d["value"]) and d["value"] > 0
    for o in outs[1:]:
        assert not any(ln.startswith("{") for ln in o.splitlines())
    (tmp_path / "bench.json").write_text(lines[0])
    print(f"bench --gpus {world} ({solver}) on one GPU over sockets: {d['value']} {d['unit']}")
