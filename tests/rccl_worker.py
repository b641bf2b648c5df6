"""One rank of the cross-process RCCL check (tests/test_gpu_rccl_procs.py); not a test module itself.

Run as a process per rank (RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT in the environment), all ranks on
GPU 0 of a one-GPU box. RCCL refuses two ranks on one device of one host ("Duplicate GPU detected"); each
rank therefore gets its own NCCL_HOSTID, so RCCL treats the ranks as separate hosts and connects them
through its socket transport on the loopback interface. What runs is the product's multi-process path as
the driver's N-GPU bench runs it — gloo for the control plane, the RCCL unique id broadcast through
torch.distributed, `lbf_comm_init(ctx, world, rank, id)`, and `ncclAllReduce` inside every data-parallel
evaluation — only the wire differs (sockets instead of xGMI). The parent test compares the results with the
in-process rank group (lbf_comm_init_local) at the same world size, bitwise at world 2 (a sum of two fp32
terms does not depend on the order), and with the single route within fp32 rounding.

argv: <output prefix>. Writes <prefix>.rank<r>.npz.
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import __graft_entry__  # noqa: E402

CFG2 = ([784, 128, 10], ["relu", "linear"], 60000)
SLB = ([784, 16, 10], ["relu", "linear"], 512)
SLB_ARGS = dict(M=5, L=4, b=32, b_H=16, step=0.02, max_epochs=2, tol=0.0, lam=1e-4)


def shard(N, world, r):
    return N * r // world, N * (r + 1) // world


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()


def allreduce_input(rank):
    return torch.randn(100003, generator=torch.Generator().manual_seed(7 + rank))


def run_rank(pkg, ctx, rank, world):
    """Every product call of the check, as one rank. Shared with the parent's rank-group run (same calls
    on a context of lbf_comm_init_local), so both sides run the same sequence."""
    res = {}
    buf = allreduce_input(rank).cuda()
    ctx.allreduce_(buf)
    res["allreduce"] = buf.cpu().numpy()
    dims, acts, N = CFG2
    Xh, Yh = pkg.synth_mnist(N)
    lo, hi = shard(N, world, rank)
    X, Y = dev(Xh[lo:hi]), dev(Yh[lo:hi])
    net = pkg.Mlp(ctx, dims, acts)
    P0 = net.init_params(123, "cpu")
    loss, g = net.loss_grad(P0, X, Y, inv_scale=1.0 / N)
    res["cfg2_loss"] = np.float64(loss)
    res["cfg2_grad"] = g.cpu().numpy()
    for ls in ("wolfe", "armijo"):
        P = P0.clone()
        h, info = pkg.lbfgs_solve(net, P, X, Y, n_global=N, line_search=ls, m=10, max_iters=10, tol=0.0)
        res[f"{ls}_loss"] = np.asarray(h["loss"])
        res[f"{ls}_trials"] = np.asarray(h["ls_trials"])
        res[f"{ls}_accepted"] = np.asarray(h["accepted"])
        res[f"{ls}_P"] = P.cpu().numpy()
        res[f"{ls}_rows"] = np.int64(info.n_rows)
    dims, acts, N = SLB
    Xh, Yh = pkg.synth_mnist(N)
    X, Y = dev(Xh), dev(Yh)
    snet = pkg.Mlp(ctx, dims, acts)
    S0 = snet.init_params(123, "cpu")
    for mode in ("sliced", "replicated"):
        P = S0.clone()
        h, _ = pkg.slbfgs_solve(snet, P, X, Y, dp_mode=mode, **SLB_ARGS)
        res[f"slbfgs_{mode}_loss"] = np.asarray(h["loss"])
        res[f"slbfgs_{mode}_accepted"] = np.asarray(h["accepted"])
        res[f"slbfgs_{mode}_P"] = P.cpu().numpy()
    torch.cuda.synchronize()
    return res


def main():
    out = sys.argv[1]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    pkg = __graft_entry__.load_package()
    ctx = pkg.Context(0, use_torch_stream=False)
    uid = [pkg.Context.unique_id() if rank == 0 else None]
    torch.distributed.broadcast_object_list(uid, src=0)
    ctx.comm_init(world, rank, uid[0])
    res = run_rank(pkg, ctx, rank, world)
    np.savez(f"{out}.rank{rank}.npz", **res)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()
    print(f"rank {rank} of {world}: ok", flush=True)


if __name__ == "__main__":
    main()
