"""Phase timestamps of the one-block history step at the two-loop microbenchmark's shape (debug build:
make -C lbfgs-ffnn_amd ktrace). For each m: the fold route's hist_step_kernel (m > 20) or the gram_fin
route's dir_cols_fin_kernel (m <= 20), last launch, wall-clock offsets in us (100 MHz clock).

    python profiles/r06/ktrace_hist.py [--m 10,50] [--samples 4096]
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["LBF_LIB_PATH"] = os.path.join(ROOT, "lbfgs-ffnn_amd", "build", "ktrace", "liblbfgs_amd_abi3.so")
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import __graft_entry__  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=str, default="10,50")
    ap.add_argument("--samples", type=int, default=4096)
    a = ap.parse_args()
    pkg = __graft_entry__.load_package()
    from lbfgs_ffnn_amd import _lib  # noqa
    L = _lib.lib()
    L.lbf_dbg_ktrace.argtypes = [C.c_void_p, C.c_int]
    L.lbf_dbg_ktrace_dir.argtypes = [C.c_void_p, C.c_int]
    ctx = pkg.Context(0)
    dims = [4096, 2048, 1024, 1]
    net = pkg.Mlp(ctx, dims, ["relu", "relu", "linear"])
    g = torch.Generator(device="cuda").manual_seed(123)
    X = torch.randn(a.samples, dims[0], device="cuda", generator=g)
    v = torch.randn(dims[0], 1, device="cuda", generator=g)
    Y = (torch.tanh(X @ v / 64.0) + 0.01 * torch.randn(a.samples, 1, device="cuda", generator=g)).contiguous()
    for m in [int(x) for x in a.m.split(",")]:
        P = net.init_params(123, "cpu")
        run = pkg.LbfgsRun(net, P, X.contiguous(), Y, m=m, max_iters=1 << 30, tol=0.0)
        run.iterate(m + 4)
        torch.cuda.synchronize()
        buf = (C.c_ulonglong * 80)()
        dbuf = (C.c_ulonglong * 80)()
        assert L.lbf_dbg_ktrace(buf, 80) == 0 and L.lbf_dbg_ktrace_dir(dbuf, 80) == 0
        run.close()
        if m > 20:
            src, t0 = buf, buf[0]
            marks = [("prefetch+prologue", 1), ("column sums", 2)]
        else:
            src, t0 = dbuf, dbuf[49]
            marks = [("last block arrives", 50), ("dots+SY/YY landed", 51)]
        marks += [("hist_core start", 56), ("push decided", 57), ("staged", 59), ("bwd start", 63),
                  ("bwd end", 60), ("fwd end", 61), ("coef stored", 62)]
        print(f"m={m} ({'hist_step' if m > 20 else 'dir_cols_fin'}):",
              "  ".join(f"{n} {(src[i] - t0) / 100.0:.2f}" for n, i in marks if src[i] >= t0), flush=True)


if __name__ == "__main__":
    main()
