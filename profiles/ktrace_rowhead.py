"""Phase timestamps of the S-LBFGS row head (debug build: make -C lbfgs-ffnn_amd ktrace), block 0 / thread 0
of the last launch, on config 4's minibatch evaluation (784-512-256-10, b = 256 rows: split-K forward, row
head over the last hidden layer's slabs). Offsets in us from the kernel's entry:
  41 staging + first-row loads issued, 42 landed (LDS barrier), 43 row sums, 44 Z / loss / dZ,
  45 delta + LDS partial (row loop done), 46 partials barrier, 47 slab written."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["LBF_LIB_PATH"] = os.path.join(ROOT, "lbfgs-ffnn_amd", "build", "ktrace", "liblbfgs_amd_abi3.so")
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import __graft_entry__  # noqa: E402


def main():
    pkg = __graft_entry__.load_package()
    from lbfgs_ffnn_amd import _lib  # noqa
    L = _lib.lib()
    ctx = pkg.Context(0)
    dims, acts = [784, 512, 256, 10], ["relu", "relu", "linear"]
    Xh, Yh = pkg.synth_mnist(256, 784, 10, 7)
    X, Y = torch.from_numpy(Xh).cuda(), torch.from_numpy(Yh).cuda()
    net = pkg.Mlp(ctx, dims, acts)
    P = net.init_params(123, "cpu")
    L.lbf_dbg_ktrace_head.argtypes = [C.c_void_p, C.c_int]
    names = {41: "loads issued", 42: "landed", 43: "row sums", 44: "Z/loss/dZ", 45: "delta+partial",
             46: "barrier", 47: "slab written"}
    for rep in range(5):
        for _ in range(20):
            net.loss_grad(P, X, Y, inv_scale=1.0 / 256)
        torch.cuda.synchronize()
        buf = (C.c_ulonglong * 64)()
        assert L.lbf_dbg_ktrace_head(buf, 64) == 0
        t0 = buf[40]
        print(f"rep {rep}: " + "  ".join(f"{names[i]} {(buf[i] - t0) / 100.0:.2f}" for i in range(41, 48)))


if __name__ == "__main__":
    main()
