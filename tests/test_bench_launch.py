"""bench.py's multi-rank entry on CPU (no GPU is touched):

* the launch decision: `bench.py --gpus N` with no WORLD_SIZE starts N rank processes (rank r on GPU r,
  rendezvous on 127.0.0.1), refuses loudly when fewer than N GPUs are visible, and runs in-process when
  torch.distributed.run already made it a rank;
* the children supervisor: exit code of the job, a failing rank takes the others down;
* the world-2 control plane of `run_rank` under gloo — RCCL unique-id broadcast, the dominant-section
  broadcast, the barriers around the timed region, the MAX of the ranks' clocks and rank-0-only emission —
  driven with a host stub of the engine whose per-iteration "all-reduce" is staged through gloo.
"""
import json
import os
import subprocess
import sys
import tempfile
import time
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_launch_plan_single_rank_cases():
    assert bench.launch_plan(1, {}, [], 0) is None                       # default: this process
    assert bench.launch_plan(4, {"WORLD_SIZE": "4"}, ["--gpus", "4"], 0) is None   # torchrun child
    assert bench.launch_plan(1, {"WORLD_SIZE": "4"}, [], 0) is None
    with pytest.raises(SystemExit, match="WORLD_SIZE=4"):
        bench.launch_plan(2, {"WORLD_SIZE": "4"}, ["--gpus", "2"], 8)


def test_launch_plan_spawns_one_rank_per_gpu():
    argv = ["--gpus", "4", "--steps", "7"]
    plan = bench.launch_plan(4, {"PATH": "/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}, argv, 8)
    assert len(plan) == 4
    ports = {e["MASTER_PORT"] for _, e in plan}
    assert len(ports) == 1
    for r, (cmd, e) in enumerate(plan):
        assert cmd[0] == sys.executable and cmd[1].endswith("bench.py") and cmd[2:] == argv
        assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"]) == (str(r), str(r), "4")
        assert e["MASTER_ADDR"] == "127.0.0.1"
        assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e["PATH"] == "/bin"


def test_launch_plan_refuses_missing_gpus():
    with pytest.raises(SystemExit, match="needs 8 visible GPUs"):
        bench.launch_plan(8, {}, ["--gpus", "8"], 1)


def test_bench_gpus2_without_gpus_fails_loudly():
    """The real entry point on this GPU-less host: non-zero exit, a clear message, no JSON line."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "needs 2 visible GPUs" in r.stderr
    assert r.stdout.strip() == ""


def test_run_children_exit_codes():
    ok = [([sys.executable, "-c", "pass"], dict(os.environ))] * 2
    assert bench.run_children(ok, poll_s=0.05) == 0
    # one rank fails fast while the other would wait forever (a rank stuck in a barrier): the job ends
    # with the failing rank's code and the waiting rank is terminated
    plan = [([sys.executable, "-c", "import sys; sys.exit(3)"], dict(os.environ)),
            ([sys.executable, "-c", "import time; time.sleep(120)"], dict(os.environ))]
    t0 = time.time()
    assert bench.run_children(plan, poll_s=0.05, grace_s=5.0) == 3
    assert time.time() - t0 < 30


# ---- world-2 control plane with a host stub of the engine ---------------------------------------------

class _Info:
    def __init__(self):
        self.n_evals = 0
        self.n_loss_only = 0
        self.n_grad_after_loss = 0
        self.n_rows = 0
        self.iterations = 0
        self.final_loss = 0.5


class _Ctx:
    uid_seen = None

    def __init__(self, dev):
        self.dev = dev
        self.sel, self.on, self.times, self.work = None, False, {}, {}

    @staticmethod
    def unique_id():
        return os.urandom(128)

    def comm_init(self, world, rank, uid):
        _Ctx.uid_seen = (world, rank, bytes(uid))

    def prof_select(self, name):
        self.sel = name

    def prof_sample(self, k):
        pass

    def prof_enable(self, on):
        self.on = on
        if on:
            self.times, self.work = {}, {}

    def prof_read(self):
        return dict(self.times)

    def prof_read_work(self):
        return dict(self.work)

    def record(self, name, ms, rows):
        if self.on and (self.sel is None or self.sel == name):
            t, c = self.times.get(name, (0.0, 0))
            self.times[name] = (t + ms, c + 1)
            self.work[name] = self.work.get(name, 0.0) + rows


class _Net:
    def __init__(self, ctx, dims, acts):
        self.ctx, self.dims = ctx, dims
        self.n = sum((dims[i] + 1) * dims[i + 1] for i in range(len(dims) - 1))

    def init_params(self, seed, init):
        return torch.zeros(self.n)

    def new_params(self):
        return torch.zeros(self.n)

    def loss_grad(self, P, X, Y, inv_scale=None, grad=None):
        # bench's device warm-up: the same count on every rank, each evaluation one collective (the DP route)
        g = torch.ones(4, dtype=torch.float64)
        dist.all_reduce(g)
        self.warm = getattr(self, "warm", 0) + 1
        return 0.0, grad


class _Run:
    """Stands in for LbfgsRun / SlbfgsRun: every iteration all-reduces a rank-tagged vector through gloo (the
    data path's one collective per evaluation) and records two kernel sections; the rank's breakdown makes a
    DIFFERENT section dominant on rank 1, so rank 1 must adopt rank 0's choice from the broadcast."""

    def __init__(self, net, P, X, Y, **kw):
        self.net, self.kw, self.rows = net, kw, X.shape[0]
        self.hist = types.SimpleNamespace(size=0)
        self.info = _Info()
        self.rank, self.world = dist.get_rank(), dist.get_world_size()

    def iterate(self, k):
        for _ in range(k):
            g = torch.full((8,), float(self.rank + 1), dtype=torch.float64)
            dist.all_reduce(g)
            assert float(g[0]) == self.world * (self.world + 1) / 2
            big = "gemm_fwd[0]" if self.rank == 0 else "gemm_dw[0]"
            small = "gemm_dw[0]" if self.rank == 0 else "gemm_fwd[0]"
            self.net.ctx.record(big, 0.2, self.rows)
            self.net.ctx.record(small, 0.1, self.rows)
            time.sleep(0.002 * (1 + 4 * self.rank))  # rank 1 is the slow one: the job's clock is its clock
            self.hist.size += 1
            self.info.n_evals += 1
            self.info.n_rows += self.rows
            self.info.iterations += 1
        return self.info

    def close(self):
        pass


def _fake_pkg():
    def synth_mnist(N, In=784, Out=10, seed=123):
        X = np.arange(N, dtype=np.float32)[:, None].repeat(In, 1)  # row r holds r: shards are checkable
        return X, np.zeros((N, Out), np.float32)

    return types.SimpleNamespace(Context=_Ctx, Mlp=_Net, LbfgsRun=_Run, SlbfgsRun=_Run, synth_mnist=synth_mnist,
                                 grad_flops_per_sample=lambda dims: 409088.0)


def _rank_worker(rank, world, port, outdir, argv):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bench.DEV = types.SimpleNamespace(synchronize=lambda: None, set_device=lambda i: None, upload=lambda t: t)
    lines = []
    bench.emit = lines.append
    seen = {}
    real_run = _Run.__init__

    def spy(self, net, P, X, Y, **kw):
        seen.update(rows=int(X.shape[0]), first=float(X[0, 0]), kw={k: v for k, v in kw.items()
                                                                     if isinstance(v, (int, float, str))})
        real_run(self, net, P, X, Y, **kw)

    _Run.__init__ = spy
    a = bench.parse(argv)
    t0 = time.perf_counter()
    bench.run_rank(a, world, rank, rank, _fake_pkg())
    wall = time.perf_counter() - t0
    dist.destroy_process_group()
    with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
        json.dump(dict(lines=lines, seen=seen, uid=list(_Ctx.uid_seen[2]), wr=_Ctx.uid_seen[:2], wall=wall), f)


@pytest.mark.parametrize("solver", ["lbfgs", "slbfgs"])
def test_control_plane_world2_gloo(solver):
    world, port = 2, bench.free_port()
    argv = ["--gpus", "2", "--steps", "12", "--warmup", "2", "--samples", "600", "--solver", solver]
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rank_worker, args=(world, port, d, argv), nprocs=world, join=True)
        r = [json.load(open(os.path.join(d, f"r{i}.json"))) for i in range(world)]
    # the library's communicator was created from ONE unique id, broadcast from rank 0
    assert r[0]["uid"] == r[1]["uid"] and r[0]["wr"] == [2, 0] and r[1]["wr"] == [2, 1]
    # exactly one JSON line, from rank 0
    assert len(r[0]["lines"]) == 1 and r[1]["lines"] == []
    line = r[0]["lines"][0]
    assert line["n_gpus"] == 2 and line["config"]["parallelism"].startswith("dp2")
    # rank 0's dominant section (gemm_fwd) is the timed one on every rank, not rank 1's own (gemm_dw)
    assert line["roofline"]["kernel"] == "gemm_fwd[0]"
    # the job's clock is the slow rank's: >= 12 iterations x 10 ms
    assert line["ms_per_step"] >= 10.0
    assert "cpu_baseline" not in line
    if solver == "lbfgs":
        # contiguous shards of the 600 rows
        assert r[0]["seen"]["rows"] == 300 and r[1]["seen"]["rows"] == 300
        assert r[0]["seen"]["first"] == 0.0 and r[1]["seen"]["first"] == 300.0
        assert r[0]["seen"]["kw"]["n_global"] == 600
        assert line["steps"] == 12
    else:
        assert r[0]["seen"]["rows"] == 600  # S-LBFGS: every rank holds all rows, evaluates its slice
