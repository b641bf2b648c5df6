"""Phase timestamps of the small kernels (debug build: make -C lbfgs-ffnn_amd ktrace).
Runs cfg-2 L-BFGS iterations and prints, per instrumented kernel, the wall-clock offsets (us) of
its phase marks (thread 0 of block 0, last launch)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["LBF_LIB_PATH"] = os.path.join(ROOT, "lbfgs-ffnn_amd", "build", "ktrace", "liblbfgs_amd_abi3.so")
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401
import __graft_entry__  # noqa: E402

GROUPS = {"hist_step": range(0, 9), "gram(block0)": range(16, 20), "reduce_fin": range(32, 36),
          "tail_fin": [40, 45, 46, 41, 42, 43, 44], "tail_reduce(block0)": range(48, 55),
          "hist_core(in tail_fin)": range(56, 63)}


def main():
    pkg = __graft_entry__.load_package()
    from lbfgs_ffnn_amd import _lib  # noqa
    L = _lib.lib()
    ctx = pkg.Context(0)
    Xh, Yh = pkg.synth_mnist(int(os.environ.get("KT_N", "60000")))
    X, Y = torch.from_numpy(Xh).cuda(), torch.from_numpy(Yh).cuda()
    net = pkg.Mlp(ctx, [784, 128, 10], ["relu", "linear"])
    P = net.init_params(123, "cpu")
    run = pkg.LbfgsRun(net, P, X, Y, m=10, max_iters=1 << 20, tol=0.0)
    run.iterate(15)
    os.environ["LBF_SPEC_DEPTH"] = "0"  # the host-driven path for the classic kernels
    run = pkg.LbfgsRun(net, P, X, Y, m=10, max_iters=1 << 20, tol=0.0)
    run.iterate(15)
    buf = (C.c_ulonglong * 80)()
    tbuf = (C.c_ulonglong * 80)()
    L.lbf_dbg_ktrace.argtypes = [C.c_void_p, C.c_int]
    L.lbf_dbg_ktrace_tail.argtypes = [C.c_void_p, C.c_int]
    assert L.lbf_dbg_ktrace(buf, 80) == 0 and L.lbf_dbg_ktrace_tail(tbuf, 80) == 0
    for i in range(40, 64):
        buf[i] = tbuf[i]
    wall = (tbuf[60] - tbuf[63]) / 100.0
    cyc = tbuf[65] - tbuf[64]
    print(f"backward sweep: {wall:.2f} us wall, {cyc} shader cycles -> {cyc / max(wall, 1e-9):.0f} MHz")
    blk = (C.c_ulonglong * 8192)()
    L.lbf_dbg_ktrace_tail_blk.argtypes = [C.c_void_p]
    assert L.lbf_dbg_ktrace_tail_blk(blk) == 0
    nb = 1024
    # blocks that ran (a launch of fewer than 1024 blocks leaves the rest of the table zero)
    ran = [i for i in range(nb) if blk[i] and blk[4 * 1024 + i]]
    S = [[blk[k * 1024 + i] for i in ran] for k in range(5)]
    nb = len(ran)
    t0 = min(S[0])
    q = lambda v: sorted(v)[len(v) // 2]
    names = ["header", "loads", "wave0 dots", "gram sweep"]
    st = [(x - t0) / 100 for x in S[0]]
    line = [f"start {min(st):.2f}/{q(st):.2f}/{max(st):.2f}"]
    for k in range(1, 5):
        d = [(S[k][i] - S[k - 1][i]) / 100 for i in range(nb)]
        line.append(f"{names[k-1]} {min(d):.2f}/{q(d):.2f}/{max(d):.2f}")
    en = [(x - t0) / 100 for x in S[4]]
    line.append(f"end {min(en):.2f}/{q(en):.2f}/{max(en):.2f}")
    print("tail_reduce blocks 0..1023 (min/med/max us):", "  ".join(line))
    hi = [i for i in range(1024) if blk[5 * 1024 + i] > t0 and blk[6 * 1024 + i] > blk[5 * 1024 + i]]
    if hi:
        s2 = [(blk[5 * 1024 + i] - t0) / 100 for i in hi]
        e2 = [(blk[6 * 1024 + i] - t0) / 100 for i in hi]
        print(f"tail_reduce blocks >=1024 ({len(hi)}): start {min(s2):.2f}/{q(s2):.2f}/{max(s2):.2f}  "
              f"end {min(e2):.2f}/{q(e2):.2f}/{max(e2):.2f}")
    # the tail's timeline on its last launch, from the first tail_reduce block's start
    endr = max(x for x in S[4] if x) if any(S[4]) else 0
    marks = [("reduce end (last block)", endr), ("cols_fin block0 start", tbuf[39]), ("fin start", tbuf[40]),
             ("fin prefetch issued", tbuf[45]), ("fin loads landed", tbuf[46]), ("decision", tbuf[41]),
             ("hist prologue", tbuf[42]), ("hist_core start", tbuf[56]), ("push", tbuf[57]),
             ("staged", tbuf[59]), ("bwd loop start", tbuf[63]), ("bwd loop end", tbuf[60]), ("fwd loop end", tbuf[61]),
             ("coef stored", tbuf[62]), ("fin end", tbuf[44])]
    print("tail timeline (us from the first tail_reduce block's start):",
          "  ".join(f"{n} {(v - t0) / 100:.2f}" for n, v in marks if v))
    for name, rg in GROUPS.items():
        t0 = buf[rg[0]]
        print(name, " ".join(f"{(buf[i] - t0) / 100.0:.2f}" for i in rg))


if __name__ == "__main__":
    main()
