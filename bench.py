"""Benchmark: full-batch L-BFGS iterations/s on the BASELINE.json headline workload.

Workload (BASELINE.json configs[1]): 784-128-10 MLP (ReLU, Linear), full-batch L-BFGS m=10 with the
reference's CPU semantics (Wolfe line search, lbfgs.hpp:38-100), N = 60000 synthetic MNIST-shaped
samples (SURVEY.md §8(d) recipe), fp32, tolerance 0 (fixed iteration count). A "step" = one L-BFGS
iteration (two-loop direction + line-search trials, each a fused loss+grad evaluation).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

With N > 1 the 60000 samples are split into contiguous shards (strong scaling; one RCCL all-reduce
of [grad | loss] per evaluation, on the library's own communicator). The torch.distributed group is
gloo: it carries only the RCCL unique id, the barriers and the max over the ranks' clocks. Rank 0
prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

METRIC = "L-BFGS iters/sec + grad-eval GFLOP/s, 784-128-10 MLP full-batch"
REF_GPU_ITERS_PER_S = 139.1      # L-BFGS m=10, 784-128-10, N=60000 (sm_86, fp32 cuBLAS)
# BASELINE.md's published GPU L-BFGS rates (the reference's CUDA route, N = 60000), by (dims, m)
REF_GPU = {("784,128,10", 10): 139.1, ("784,128,10", 100): 87.2,
           ("784,256,128,64,10", 10): 60.7, ("784,256,128,64,10", 100): 51.6}
FP32_MFMA_PEAK_TFLOPS = 157.3    # MI355X_MICROARCH.md: FP32 matrix peak (dense)
HBM_PEAK_GBS = 8000.0
PROF_EVERY = 8                   # time every 8th launch of the dominant kernel inside the timed region ...
PROF_MIN_LAUNCHES = 10           # ... or more often, so that at least this many launches are timed (an event
                                 # pair costs ~10 us of GPU time: profiles/r03/launch_floor.txt)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 400 iterations (~0.12 s at cfg 2): a few-ms host stall of the speculating thread (a shared box) is a
    # few percent of the timed region instead of >10 % at 100
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--samples", type=int, default=60000)
    ap.add_argument("--dims", type=str, default="784,128,10")
    ap.add_argument("--acts", type=str, default="relu,linear")
    ap.add_argument("--m", type=int, default=10)
    ap.add_argument("--line-search", type=str, default="wolfe",
                    help="wolfe: the reference's CPU semantics (lbfgs.hpp:38-100); armijo: its CUDA semantics "
                         "(lbfgs.cuh:39-194), the route its published GPU it/s were measured on")
    ap.add_argument("--init", choices=["cpu", "cuda"], default="cpu",
                    help="parameter-init stream: cpu = network.hpp:45-71 (all params N(0, s)), cuda = "
                         "network.cuh:36-59 (weights N(0, s), zero biases; the reference's GPU drivers)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--device-warmup", type=int, default=300,
                    help="L-BFGS: loss/gradient evaluations at the initial point before the run starts (untimed, the "
                         "same count on every rank; they leave the run's trajectory unchanged): the chip reaches its "
                         "steady clock before the breakdown pass and the timed iterations (profiles/r04/l/drv_*.json)")
    ap.add_argument("--breakdown-last", action="store_true",
                    help="L-BFGS: run the per-section breakdown pass after the warmup iterations (the round-2/3 "
                         "order) instead of before them")
    ap.add_argument("--comm1", action="store_true",
                    help="at N=1, route evaluations through a 1-rank RCCL communicator (the DP code path)")
    ap.add_argument("--cpu-iters", type=int, default=64)  # at most; a probe bounds each run to CPU_BUDGET_S
    ap.add_argument("--cpu-samples", type=int, default=0,
                    help="rows of the CPU-baseline sample (0: all rows up to 60000, else 2000; scaled to N)")
    ap.add_argument("--data", choices=["mnist", "regression"], default="mnist",
                    help="mnist: SURVEY §8(d) MNIST-shaped classes (configs 1-4); regression: config 5's "
                         "device-generated X ~ N(0,1), y = tanh(v.x/64) + 0.01 e")
    ap.add_argument("--pmc-json", type=str, default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--solver", choices=["lbfgs", "slbfgs"], default="lbfgs",
                    help="slbfgs: BASELINE config 4 (S-LBFGS 784-512-256-10, b=256, b_H=128, L=M=10); a step "
                         "is one epoch")
    ap.add_argument("--slbfgs-b", type=int, default=256, help="S-LBFGS minibatch b (config 4: 256)")
    ap.add_argument("--slbfgs-bh", type=int, default=128, help="S-LBFGS Hessian batch b_H (config 4: 128)")
    ap.add_argument("--slbfgs-dp", choices=["replicated", "sliced"], default="replicated",
                    help="S-LBFGS over N > 1 ranks: replicated = every rank runs the whole minibatch chain, only the "
                         "epoch's full-batch gradient is sharded (one all-reduce per epoch); sliced = each rank "
                         "evaluates 1/N of every minibatch (one all-reduce per inner step)")
    ap.add_argument("--slbfgs-step", type=float, default=0.005,
                    help="S-LBFGS step (config 4 names 0.02, which diverges to NaN on the synthetic data in the "
                         "fp64 oracle too; the work per epoch does not depend on it)")
    a = ap.parse_args(argv)
    if a.solver == "slbfgs" and a.dims == "784,128,10":
        a.dims, a.acts = "784,512,256,10", "relu,relu,linear"
    return a


def host_cpu():
    """CPU model and core counts of this host (/proc/cpuinfo, the data lscpu prints)."""
    model, cores = None, set()
    try:
        phys = core = None
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name" and model is None:
                model = v
            elif k == "physical id":
                phys = v
            elif k == "core id":
                core = v
            elif not k and phys is not None:
                cores.add((phys, core))
                phys = core = None
        if phys is not None:
            cores.add((phys, core))
    except OSError:
        pass
    return dict(model=model, physical_cores=len(cores) or None, logical_cpus=os.cpu_count(),
                usable_cpus=len(os.sched_getaffinity(0)))


def route_env():
    """LBF_* variables that reroute kernels (tests and A/B builds use them); reported in the bench line so
    a stray one cannot change the measured route without a trace."""
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith("LBF_")}


def cgroup_cpus():
    """CPUs the job's cgroup may use (cpu.max quota / period), or None when unlimited / unknown."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else round(q / p, 2)
    except (OSError, ValueError):
        return None


THREADS_NOTE = ("value: OpenMP threads = the CPUs this job may use: the host's physical cores, capped by the "
                "job's cgroup CPU quota (16 of the 128 physical cores on the GPU box; OMP_NUM_THREADS is 16 there "
                "too); at_physical_cores: the same oracle at one thread per physical core (BASELINE.md §2), which "
                "on the GPU box oversubscribes the 16-CPU quota and runs slower; the reference's own CPU numbers "
                "(BASELINE.md) do not state their thread count")
CPU_BUDGET_S = 30.0   # bound on the primary CPU-baseline run (the sample shrinks when a probe predicts more)
CPU_BUDGET_PHYS_S = 15.0   # bound on the physical-core run


def baseline_threads(O):
    """(usable threads, physical-core threads, host info) for the CPU baseline's two runs."""
    hc = host_cpu()
    hc["cgroup_cpus"] = cgroup_cpus()
    phys = int(hc["physical_cores"] or os.cpu_count() or 1)
    usable = min(phys, int(hc["usable_cpus"] or phys))
    if hc["cgroup_cpus"]:
        usable = min(usable, max(1, int(hc["cgroup_cpus"])))
    return usable, phys, hc


def timed_threads(O, threads, fn):
    O.set_threads(threads)
    t0 = time.perf_counter()
    r = fn()
    return r, time.perf_counter() - t0


def bounded_iters(O, threads, fn2, budget, cap):
    """Iterations of an L-BFGS sample that a 2-iteration probe at `threads` predicts to fit `budget` s."""
    _, probe_s = timed_threads(O, threads, fn2)
    return int(max(4, min(cap, budget / max(probe_s / 2, 1e-6))))


def cpu_baseline(dims, acts, N, m, iters, data, rows):
    """The oracle (fp64 C++/OpenMP restatement of the reference CPU path, literal call pattern incl. its
    redundant f/grad re-evaluations) timed on this host at the CPUs the job may use (`value`) and at one
    thread per physical core (`at_physical_cores`); bounded sample of the same workload: `rows` of the N
    samples (the full-batch cost is linear in N, so the rate is scaled by rows / N), for as many iterations
    (at most `iters`) as a 2-iteration probe predicts to fit the run's time budget."""
    O = __graft_entry__.load_oracle()
    O.lib()
    X, Y = O.synth_mnist(rows, dims[0], dims[-1]) if data == "mnist" else O.synth_regression(rows, dims[0])
    net = O.Net(dims, acts)
    P = net.init_cpu(123)
    usable, phys, hc = baseline_threads(O)
    scale = rows / N
    probe = lambda: net.lbfgs_wolfe(P, X, Y, m=m, max_iters=2)  # noqa: E731

    def one(threads, n_it):
        (_, rec, info), _ = timed_threads(O, threads, lambda: net.lbfgs_wolfe(P, X, Y, m=m, max_iters=n_it))
        ms = info["ms"]
        return dict(value=round(n_it / (ms / 1e3) * scale, 6), cores=threads, iters=n_it,
                    seconds=round(ms / 1e3, 2), passes=f"{info['n_fwd']} forward, {info['n_bwd']} backward")

    main_run = one(usable, bounded_iters(O, usable, probe, CPU_BUDGET_S, iters))
    phys_run = one(phys, bounded_iters(O, phys, probe, CPU_BUDGET_PHYS_S, iters)) if phys != usable else None
    O.set_threads(usable)
    out = dict(value=main_run["value"], unit="iters/s", cores=usable, kind="port", host=hc, threads_note=THREADS_NOTE,
               sample=f"{main_run['iters']} L-BFGS iterations (Wolfe, m={m}) of the {'-'.join(map(str, dims))} MLP "
                      f"on {rows} of the N={N} rows{f' (rate scaled by {rows}/{N})' if rows != N else ''}, fp64 "
                      f"oracle (oracle/oracle.hpp) with the reference's f/grad call pattern ({main_run['passes']} "
                      f"passes), {usable} OpenMP threads, {main_run['seconds']} s")
    if phys_run:
        out["at_physical_cores"] = {k: phys_run[k] for k in ("value", "cores", "iters", "seconds")}
    return out


def slbfgs_cpu_baseline(dims, acts, N, step, epochs=1):
    """The oracle's S-LBFGS (fp64 restatement of s_lbfgs.hpp:165-290, OpenMP) for one epoch at full N, at the
    CPUs the job may use (an oversubscribed physical-core run of a whole epoch would take ~1 min on the GPU
    box: the cfg-2 line carries that comparison)."""
    O = __graft_entry__.load_oracle()
    X, Y = O.synth_mnist(N, dims[0], dims[-1])
    net = O.Net(dims, acts)
    P = net.init_cpu(123)
    usable, _, hc = baseline_threads(O)
    kw = dict(epochs=epochs, tol=0.0, M=10, L=10, b=256, bH=128, step=step, lam=1e-4)
    _, dt = timed_threads(O, usable, lambda: net.slbfgs(P, X, Y, **kw))
    out = dict(value=round(epochs / dt, 6), unit="epochs/s", cores=usable, kind="port", host=hc,
               threads_note=THREADS_NOTE,
               sample=f"{epochs} S-LBFGS epoch(s) of the {'-'.join(map(str, dims))} MLP on all N={N} rows (b=256, "
                      f"b_H=128, L=M=10), fp64 oracle (oracle/oracle.hpp), {usable} OpenMP threads, {dt:.1f} s")
    O.set_threads(usable)
    return out


class Device:
    """The three torch.cuda calls the rank code makes. tests/test_bench_launch.py swaps in a host stub so
    that the multi-rank control plane (unique-id broadcast, dominant-section broadcast, barriers, the MAX
    of the ranks' clocks, rank-0 emission) runs on CPU under gloo."""
    synchronize = staticmethod(lambda: torch.cuda.synchronize())
    set_device = staticmethod(lambda i: torch.cuda.set_device(i))
    upload = staticmethod(lambda t: t.cuda())


DEV = Device()
_JSON_OUT = None


def emit(line: dict):
    """The one stdout line. Everything else the process prints (RCCL's version banner at communicator
    init, libdrm notices, C printf from any library) was sent to stderr by isolate_stdout()."""
    out = _JSON_OUT or sys.stdout
    out.write(json.dumps(line) + "\n")
    out.flush()


def isolate_stdout():
    """Keep stdout for the JSON line alone: duplicate fd 1 for emit(), then point fd 1 at stderr."""
    global _JSON_OUT
    sys.stdout.flush()
    _JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)


def main_slbfgs(a, pkg, ctx, world, rank):
    """BASELINE config 4: S-LBFGS epochs/s (+ grad-evals/s); every rank holds all N rows and evaluates its
    1/world slice of each minibatch, Hessian batch and full-gradient anchor (s_lbfgs.hpp:165-290)."""
    dims = [int(x) for x in a.dims.split(",")]
    acts = a.acts.split(",")
    N = a.samples
    Xh, Yh = pkg.synth_mnist(N, dims[0], dims[-1], 123)
    X, Y = DEV.upload(torch.from_numpy(Xh)), DEV.upload(torch.from_numpy(Yh))
    del Xh, Yh
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    kw = dict(M=10, L=10, b=a.slbfgs_b, b_H=a.slbfgs_bh, step=a.slbfgs_step, lam=1e-4, tol=0.0, dp_mode=a.slbfgs_dp)
    # one stateful solve for the breakdown, the warmup and the timed epochs
    run = pkg.SlbfgsRun(net, P, X, Y, **kw)
    # first epoch with every kernel section timed: the breakdown and the dominant section
    ctx.prof_select(None)
    ctx.prof_sample(1)
    ctx.prof_enable(True)
    run.iterate(1)
    breakdown = ctx.prof_read()
    ctx.prof_enable(False)
    wep = 1
    # the dominant GEMM section (the roofline is a GEMM's); at many ranks the epoch's all-reduce can take longer,
    # but it runs once or twice per epoch, too rarely to sample
    gemms = {k: v for k, v in breakdown.items() if k.split("[")[0] in ("gemm_fwd", "gemm_dw", "gemm_dx")}
    dominant = max((gemms or breakdown).items(), key=lambda kv: kv[1][0])[0]
    if world > 1:
        obj = [dominant]
        torch.distributed.broadcast_object_list(obj, src=0)
        dominant = obj[0]
    # timed region: only the dominant section carries events, on every PROF_EVERY-th launch (an event pair
    # costs ~10 us of GPU time, and this section runs ~2x per inner step) while that still times
    # PROF_MIN_LAUNCHES of them; the rows of every timed launch are counted (lbf_prof_read_work), so the
    # sampled flops are exact whatever the batch sizes
    every = max(1, min(PROF_EVERY, int(breakdown[dominant][1] * max(a.steps, 1) // PROF_MIN_LAUNCHES)))
    ctx.prof_select(dominant)
    ctx.prof_sample(every)
    ctx.prof_enable(True)
    run.iterate(a.warmup)
    ctx.prof_enable(True)          # clears the warmup's timings
    evals0, rows0, ep0 = float(run.info.n_evals), float(run.info.n_rows), int(run.info.iterations)
    DEV.synchronize()
    if world > 1:
        torch.distributed.barrier()
    DEV.synchronize()
    t0 = time.perf_counter()
    info = run.iterate(a.steps)
    DEV.synchronize()
    elapsed = time.perf_counter() - t0
    cnt = torch.tensor([elapsed, float(info.n_evals) - evals0, float(info.n_rows) - rows0], dtype=torch.float64)
    if world > 1:
        mx = cnt[:1].clone()
        torch.distributed.all_reduce(mx, op=torch.distributed.ReduceOp.MAX)
        torch.distributed.all_reduce(cnt, op=torch.distributed.ReduceOp.SUM)
        cnt[0] = mx[0]
        torch.distributed.barrier()
    elapsed, evals_all, rows_all = float(cnt[0]), float(cnt[1]), float(cnt[2])
    prof = ctx.prof_read()
    work = ctx.prof_read_work()
    ctx.prof_enable(False)
    ctx.prof_select(None)
    ctx.prof_sample(1)
    if rank == 0:
        epochs = int(info.iterations) - ep0
        F = pkg.grad_flops_per_sample(dims)
        if dominant not in prof:
            raise SystemExit(f"bench.py: the dominant section {dominant} did not run in the timed region")
        name, (ms, launches) = dominant, prof[dominant]
        kind, layer = name.split("[")[0], int(name.split("[")[1].rstrip("]"))
        roof = dict(bound="mfma", achieved=None, peak=FP32_MFMA_PEAK_TFLOPS, unit="TFLOP/s", frac=None)
        if kind in ("gemm_fwd", "gemm_dw", "gemm_dx"):
            # algorithmic flops of the timed launches (2 In Out per row, rows counted per launch) / their
            # summed event time
            flops = 2.0 * dims[layer] * dims[layer + 1] * float(work.get(dominant, 0.0))
            roof["achieved"] = round(flops / (ms / 1e3) / 1e12, 3)
            roof["frac"] = round(roof["achieved"] / roof["peak"], 4)
        roof.update(kernel=name, avg_launch_us=round(ms * 1e3 / launches, 2), timed_launches=launches,
                    sampled_every=every, avg_rows_per_timed_launch=round(work.get(dominant, 0.0) / launches, 1),
                    traffic=pmc_traffic(a.pmc_json, name, f"{','.join(str(d) for d in dims)}:{a.samples}:{world}"))
        # (traffic: the median over the section's minibatch launches, the PMC pass's most frequent size)
        out = {
            "metric": "S-LBFGS epochs/s + grad-evals/s, 784-512-256-10 MLP",
            "value": round(epochs / elapsed, 4),
            "unit": "epochs/s",
            "n_gpus": world,
            "steps": epochs,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / max(epochs, 1) * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic",
            "config": {"workload": f"{a.dims} MLP ({a.acts}), S-LBFGS b={a.slbfgs_b} b_H={a.slbfgs_bh} L=M=10 step "
                                   f"{a.slbfgs_step} lambda 1e-4, N={N}; a step = one epoch ({N // a.slbfgs_b} inner "
                                   f"steps + the closing full-batch gradient at the new anchor)",
                       "global_batch": N,
                       "parallelism": f"dp{world}" + (f"-{a.slbfgs_dp}" if world > 1 else "")},
            "grad_evals_per_s": round(evals_all / elapsed, 1),
            "grad_eval_gflops": round(rows_all * F / elapsed / 1e9, 1),
            "final_loss": float(info.final_loss),
            "roofline": roof,
            "kernel_ms_per_step": {k: round(v[0] / wep, 4) for k, v in sorted(breakdown.items())},
            "route_env": route_env(),
        }
        if world == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = slbfgs_cpu_baseline(dims, acts, N, a.slbfgs_step)
        emit(out)
    run.close()


def visible_gpus() -> int:
    """GPUs this process may use. torch.cuda.device_count() counts them without creating a HIP context,
    so the launcher below never touches the GPU itself."""
    return torch.cuda.device_count()


def free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_plan(gpus, env, argv, visible):
    """How `bench.py --gpus N` runs.

    Returns None when this process is a rank itself: N = 1, or WORLD_SIZE is set (torch.distributed.run
    launched it; WORLD_SIZE must then equal N). Otherwise N > 1 ranks are needed and this process is only
    their launcher: returns one (argv, env) per rank, rank r on GPU r, all rendezvousing on 127.0.0.1.
    Raises SystemExit with a message (never falls back to one rank) when fewer than N GPUs are visible."""
    if "WORLD_SIZE" in env:
        ws = int(env["WORLD_SIZE"])
        if gpus not in (1, ws):
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={ws}; launch one rank per GPU")
        return None
    if gpus <= 1:
        return None
    if visible < gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} needs {gpus} visible GPUs, this host shows {visible}; "
                         f"refusing to run fewer ranks")
    port = free_port()
    plan = []
    for r in range(gpus):
        e = dict(env)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus), LOCAL_WORLD_SIZE=str(gpus),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        plan.append(([sys.executable, os.path.abspath(__file__)] + list(argv), e))
    return plan


def run_children(plan, poll_s=0.2, grace_s=10.0) -> int:
    """Start the ranks, wait for all of them; the first rank to fail takes the others down (a rank left
    waiting in a barrier would otherwise hang). Returns the job's exit code (0 only if every rank exits 0).
    Rank 0's stdout (the JSON line) is this process's stdout."""
    import subprocess
    procs = [subprocess.Popen(cmd, env=env) for cmd, env in plan]
    code = 0
    try:
        while True:
            live = [p for p in procs if p.poll() is None]
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad:
                code = bad[0]
                break
            if not live:
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        t_end = time.time() + grace_s
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - time.time()))
            except Exception:
                p.kill()
                p.wait()
    if code:
        print(f"bench.py: a rank exited with status {code}", file=sys.stderr)
    return code


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    plan = launch_plan(a.gpus, os.environ, argv,
                       visible_gpus() if a.gpus > 1 and "WORLD_SIZE" not in os.environ else 0)
    if plan is not None:
        return run_children(plan)
    isolate_stdout()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # control plane only (RCCL unique id, barriers, max of the ranks' clocks): gloo over loopback, so
        # each process holds exactly one RCCL communicator, the library's own (lbf_comm_init), and the
        # data path's all-reduce is the only collective on xGMI
        DEV.set_device(local)
        torch.distributed.init_process_group("gloo")
    try:
        run_rank(a, world, rank, local, __graft_entry__.load_package())
    finally:
        if world > 1:
            torch.distributed.destroy_process_group()
    return 0


def pmc_traffic(path, section, config):
    """HBM bytes per launch of `section` for `config` from the committed PMC summary (profiles/
    pmc_traffic.json: one entry or a list of them, written by profiles/collect_pmc.py), or None."""
    if not os.path.exists(path):
        return None
    try:
        pm = json.load(open(path))
    except Exception:
        return None
    for e in pm if isinstance(pm, list) else [pm]:
        if e.get("section") == section and e.get("config") == config:
            return e.get("hbm_bytes_per_launch")
    return None


def run_rank(a, world, rank, local, pkg):
    """One rank of the benchmark (world = 1: the whole job)."""
    dims = [int(x) for x in a.dims.split(",")]
    acts = a.acts.split(",")
    N = a.samples

    ctx = pkg.Context(local)
    if world > 1:
        uid = [pkg.Context.unique_id() if rank == 0 else None]
        torch.distributed.broadcast_object_list(uid, src=0)
        ctx.comm_init(world, rank, uid[0])
    elif a.comm1:
        ctx.comm_init(1, 0, pkg.Context.unique_id())
    if a.solver == "slbfgs":
        main_slbfgs(a, pkg, ctx, world, rank)
        return
    lo, hi = N * rank // world, N * (rank + 1) // world
    if a.data == "mnist":
        Xh, Yh = pkg.synth_mnist(N, dims[0], dims[-1], 123)
        X = DEV.upload(torch.from_numpy(Xh[lo:hi]))
        Y = DEV.upload(torch.from_numpy(Yh[lo:hi]))
        del Xh, Yh
    else:  # this rank's shard generated in place
        X, Y = pkg.synth_regression(ctx, hi - lo, dims[0], row0=lo)
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, a.init)
    if a.device_warmup > 0:
        g = net.new_params()
        for _ in range(a.device_warmup):
            net.loss_grad(P, X, Y, inv_scale=1.0 / N, grad=g)
        del g
    DEV.synchronize()

    run = pkg.LbfgsRun(net, P, X, Y, n_global=N, line_search=a.line_search, m=a.m, max_iters=1 << 30, tol=0.0,
                       record_cap=a.warmup + 2 * a.steps + 28)
    if a.breakdown_last:
        run.iterate(a.warmup)
    # untimed pass with every kernel section timed: per-section breakdown and the dominant section. It runs
    # before the W warmup iterations, so that the timed region follows full-speed iterations (the
    # breakdown's event on every launch leaves the chip below its steady clock); the timed iterations are
    # the same ones either way (the breakdown's + W iterations precede them).
    ctx.prof_select(None)
    ctx.prof_enable(True)
    bd_steps = max(1, min(a.steps, 20))
    bd0 = run.hist.size
    run.iterate(bd_steps)
    breakdown = ctx.prof_read()
    bd_steps = max(run.hist.size - bd0, 1)
    ctx.prof_enable(False)
    if not a.breakdown_last:
        run.iterate(a.warmup)
    # the section with the largest total time among those that run at least once per iteration (a section of
    # the occasional non-speculative start can win the breakdown when a profiler serialises the launches)
    regular = {k: v for k, v in breakdown.items() if v[1] >= bd_steps} or breakdown
    # the roofline is a GEMM's: at many ranks the all-reduce section can take longer than any GEMM
    gemms = {k: v for k, v in regular.items() if k.split("[")[0] in ("gemm_fwd", "gemm_dw", "gemm_dx")}
    dominant = max((gemms or regular).items(), key=lambda kv: kv[1][0])[0]
    if world > 1:  # every rank must time the same section (identical launch sequences)
        obj = [dominant]
        torch.distributed.broadcast_object_list(obj, src=0)
        dominant = obj[0]
    # timed region: only the dominant kernel carries an event pair
    evals0, lonly0, gal0 = run.info.n_evals, run.info.n_loss_only, run.info.n_grad_after_loss
    it0 = run.hist.size
    ctx.prof_select(dominant)
    # the dominant section runs about once per evaluation: sample every PROF_EVERY-th launch only when
    # that still times PROF_MIN_LAUNCHES of them
    launches = breakdown[dominant][1] / max(bd_steps, 1) * a.steps
    every = max(1, min(PROF_EVERY, int(launches // PROF_MIN_LAUNCHES)))
    ctx.prof_sample(every)
    ctx.prof_enable(True)

    def barrier():
        DEV.synchronize()
        if world > 1:
            torch.distributed.barrier()
        DEV.synchronize()

    barrier()
    t0 = time.perf_counter()
    run.iterate(a.steps)
    DEV.synchronize()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    barrier()
    prof = ctx.prof_read()
    work = ctx.prof_read_work()
    ctx.prof_enable(False)
    ctx.prof_select(None)
    ctx.prof_sample(1)
    evals = run.info.n_evals - evals0
    lonly = run.info.n_loss_only - lonly0
    gal = run.info.n_grad_after_loss - gal0
    iters_done = run.hist.size - it0

    if rank == 0:
        F = pkg.grad_flops_per_sample(dims) * N            # algorithmic flops per full-batch evaluation
        Ffwd = sum(2 * dims[l] * dims[l + 1] for l in range(len(dims) - 1)) * N  # forward pass
        # forward passes: full evaluations + loss-only trials, minus the backward halves that reused a
        # loss-only trial's forward (each counted in n_evals too); backward passes: n_evals
        fwd_passes = evals - gal + lonly
        gflops = (fwd_passes * Ffwd + evals * (F - Ffwd)) / elapsed / 1e9
        # dominant kernel: largest total time in the timed region (HIP events on the library stream)
        if dominant not in prof:
            raise SystemExit(f"bench.py: the dominant section {dominant} did not run in the timed region")
        name, (ms, cnt) = dominant, prof[dominant]
        avg_s = ms / 1e3 / cnt
        kind, layer = name.split("[")[0], int(name.split("[")[1].rstrip("]"))
        n_loc = hi - lo
        In, Out = dims[layer], dims[layer + 1]
        if kind in ("gemm_fwd", "gemm_dw", "gemm_dx"):
            flops = 2.0 * In * Out * work.get(dominant, n_loc * cnt) / cnt  # per launch (rows counted), per rank
            roof = dict(bound="mfma", achieved=round(flops / avg_s / 1e12, 3), peak=FP32_MFMA_PEAK_TFLOPS,
                        unit="TFLOP/s")
        else:
            roof = dict(bound="hbm", achieved=None, peak=HBM_PEAK_GBS, unit="GB/s")
        roof["frac"] = round(roof["achieved"] / roof["peak"], 4) if roof["achieved"] else None
        roof["kernel"] = name
        roof["avg_launch_us"] = round(avg_s * 1e6, 2)
        roof["timed_launches"] = cnt
        roof["sampled_every"] = every
        roof["traffic"] = pmc_traffic(a.pmc_json, name, f"{a.dims}:{N}:{world}")
        ms_step = elapsed / max(iters_done, 1) * 1e3
        value = iters_done / elapsed
        out = {
            "metric": METRIC if a.dims == "784,128,10" else METRIC.replace("784-128-10", a.dims.replace(",", "-")),
            "value": round(value, 3),
            "unit": "iters/s",
            "n_gpus": world,
            "steps": iters_done,
            "warmup": a.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": (round(value / REF_GPU[(a.dims, a.m)], 3)
                            if N == 60000 and (a.dims, a.m) in REF_GPU else None),
            "dtype": "fp32",
            "data": "synthetic" if a.data == "mnist" else "synthetic (config-5 regression stream, device-generated)",
            "config": {"workload": f"{a.dims} MLP ({a.acts}), full-batch L-BFGS m={a.m} "
                                   f"({a.line_search} line search, "
                                   f"{'CPU' if a.line_search == 'wolfe' else 'CUDA'}-reference semantics, "
                                   f"{a.init} init stream), N={N}",
                       "global_batch": N,
                       "parallelism": f"dp{world}" + ("+rccl1" if a.comm1 and world == 1 else "")},
            "grad_eval_gflops": round(gflops, 1),
            "evals_per_iter": round(evals / max(iters_done, 1), 3),
            "loss_only_trials_per_iter": round(lonly / max(iters_done, 1), 3),
            "forward_passes_per_iter": round(fwd_passes / max(iters_done, 1), 3),
            "roofline": roof,
            "kernel_ms_per_step": {k: round(v[0] / bd_steps, 4) for k, v in sorted(breakdown.items())},
            "route_env": route_env(),
        }
        if world == 1 and not a.no_cpu_baseline:
            rows = a.cpu_samples or (N if N <= 60000 else 2000)
            out["cpu_baseline"] = cpu_baseline(dims, acts, N, a.m, a.cpu_iters, a.data, min(rows, N))
        emit(out)
    run.close()


if __name__ == "__main__":
    sys.exit(main())
