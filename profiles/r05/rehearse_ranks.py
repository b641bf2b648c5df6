"""Rehearsal of the driver's N-GPU bench command on a one-GPU box: N bench.py rank processes (WORLD_SIZE set, as
torch.distributed.run starts them), every one on GPU 0 with its own NCCL_HOSTID so RCCL connects them through its
socket transport on loopback (tests/test_gpu_rccl_procs.py). Checks that rank 0 prints one JSON line with
n_gpus N / dpN and that every rank exits 0. The rate of N ranks sharing one GPU over sockets is not a result.

    python profiles/r05/rehearse_ranks.py N [bench args...]
"""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    world = int(sys.argv[1])
    extra = sys.argv[2:]
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(world):
        e = dict(os.environ)
        e.update(RANK=str(r), LOCAL_RANK="0", WORLD_SIZE=str(world), LOCAL_WORLD_SIZE="1", GROUP_RANK=str(r),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), NCCL_HOSTID=f"lbf-rehearsal-rank{r}",
                 NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", str(world)] + extra,
                                      env=e, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, cwd=ROOT))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=600)[0])
    except subprocess.TimeoutExpired:
        for p in procs:
            p.kill()
        raise SystemExit("a rank overran 600 s")
    codes = [p.returncode for p in procs]
    lines = [ln for ln in outs[0].splitlines() if ln.startswith("{")]
    ok = all(c == 0 for c in codes) and len(lines) == 1
    if ok:
        d = json.loads(lines[0])
        ok = d["n_gpus"] == world and d["config"]["parallelism"].startswith(f"dp{world}")
        print(json.dumps({"world": world, "args": extra, "rank_exit_codes": codes, "value": d["value"],
                          "unit": d["unit"], "parallelism": d["config"]["parallelism"], "ok": ok}))
    if not ok:
        print("exit codes", codes)
        for r, o in enumerate(outs):
            print(f"--- rank {r} ---\n{o[-3000:]}")
        raise SystemExit(1)


if __name__ == "__main__":
    main()
