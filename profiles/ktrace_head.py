"""Phase stamps of the standalone head kernel (debug build: make -C lbfgs-ffnn_amd ktrace) on the S-LBFGS
minibatch shape (784-512-256-10, b = 256): wall-clock offsets (us, 100 MHz) of block 0's marks, last launch.
  30 entry | 31 W staged | 32 tile staged | 34-39 tile(): forward, loss/dZ, dW strips, delta | 33 slab written"""
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
    B = int(os.environ.get("KT_B", "256"))
    dims = [784, 512, 256, 10]
    Xh, Yh = pkg.synth_mnist(B, 784, 10)
    X, Y = torch.from_numpy(Xh).cuda(), torch.from_numpy(Yh).cuda()
    net = pkg.Mlp(ctx, dims, ["relu", "relu", "linear"])
    P = net.init_params(123, "cpu")
    buf = (C.c_ulonglong * 64)()
    L.lbf_dbg_ktrace_head.argtypes = [C.c_void_p, C.c_int]
    rows = []
    for it in range(20):
        net.loss_grad(P, X, Y, inv_scale=1.0 / B)
        torch.cuda.synchronize()
        assert L.lbf_dbg_ktrace_head(buf, 64) == 0
        t0 = buf[30]
        rows.append([(buf[i] - t0) / 100.0 for i in (31, 32, 34, 35, 36, 37, 38, 39, 33)])
    import statistics
    names = ["W staged", "tile staged", "tile start", "forward", "loss/dZ", "dW strips", "delta", "tile end", "slab"]
    med = [statistics.median(r[i] for r in rows[5:]) for i in range(len(names))]
    print("head kernel block 0 phase ends (us after entry, median of 15 launches):")
    for n, v in zip(names, med):
        print(f"  {n:12s} {v:7.2f}")


if __name__ == "__main__":
    main()
