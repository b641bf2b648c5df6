"""Block-0 timeline of the fused forward GEMM + head (debug build: make -C lbfgs-ffnn_amd ktrace)."""
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
    for N in [int(x) for x in os.environ.get("NS", "7500,60000").split(",")]:
        X = torch.randn(N, 784, device="cuda")
        Y = torch.randn(N, 10, device="cuda")
        net = pkg.Mlp(ctx, [784, 128, 10], ["relu", "linear"])
        P = net.init_params(1, "cpu")
        for _ in range(3):
            net.loss_grad(P, X, Y)
        torch.cuda.synchronize()
        buf = (C.c_ulonglong * 42)()
        L.lbf_dbg_ktrace_gemm.argtypes = [C.c_void_p, C.c_int]
        assert L.lbf_dbg_ktrace_gemm(buf, 42) == 0
        t0 = buf[0]
        its = [(buf[i] - t0) / 100.0 for i in range(1, 26)]
        print(f"N={N} k-iters end (us):", " ".join(f"{x:.2f}" for x in its))
        print(f"N={N} main loop: {buf[41] - buf[40]} shader cycles in {(buf[25] - buf[0]) / 100.0:.2f} us "
              f"-> {(buf[41] - buf[40]) / ((buf[25] - buf[0]) * 10.0):.3f} GHz")
        print(f"N={N} head epilogue end {(buf[32] - t0) / 100.0:.2f}  partials end {(buf[33] - t0) / 100.0:.2f}")
        print(f"N={N} epilogue: start {(buf[26]-t0)/100:.2f} w-staged {(buf[27]-t0)/100:.2f} "
              f"half0 staged {(buf[28]-t0)/100:.2f} done {(buf[29]-t0)/100:.2f} "
              f"half1 staged {(buf[30]-t0)/100:.2f} done {(buf[31]-t0)/100:.2f}")
        print(f"N={N} last head tile phases (us from its start):",
              " ".join(f"{(buf[i] - buf[34]) / 100.0:.2f}" for i in range(34, 40)))
        nb = min(1024, (N + 127) // 128)
        blk = (C.c_ulonglong * 8192)()
        L.lbf_dbg_ktrace_gemm_blk.argtypes = [C.c_void_p]
        assert L.lbf_dbg_ktrace_gemm_blk(blk) == 0
        S = [[blk[k * 1024 + i] for i in range(nb)] for k in range(8)]
        t0 = min(S[0])
        q = lambda v: sorted(v)[len(v) // 2]
        starts = [(x - t0) / 100 for x in S[0]]
        names = ["main loop", "w/y store", "stage h0", "tile h0", "stage h1", "tile h1", "partials"]
        line = []
        for k in range(1, 8):
            d = [(S[k][i] - S[k - 1][i]) / 100 for i in range(nb) if S[k][i] and S[k - 1][i] and S[k][i] >= S[k - 1][i]]
            if d:
                line.append(f"{names[k-1]} {min(d):.2f}/{q(d):.2f}/{max(d):.2f}")
        ends = [(x - t0) / 100 for x in S[7]]
        print(f"N={N} blocks={nb} (min/med/max us): " + "  ".join(line) + f"  end {min(ends):.2f}/{q(ends):.2f}/{max(ends):.2f}")
        late = sorted(range(nb), key=lambda i: starts[i])[-8:]
        print(f"N={N} latest starters:", " ".join(f"{i}:{starts[i]:.1f}" for i in late))
        # placement (lbf_kt_hw: XCC id, HW_ID): main loop and end by XCD and by blocks sharing the CU
        hw = (C.c_ulonglong * 1024)()
        if hasattr(L, "lbf_dbg_ktrace_gemm_hw"):
            L.lbf_dbg_ktrace_gemm_hw.argtypes = [C.c_void_p]
            assert L.lbf_dbg_ktrace_gemm_hw(hw) == 0
            key = []
            for i in range(nb):
                h = hw[i] & 0xffffffff
                key.append((hw[i] >> 32, (h >> 13) & 7, (h >> 12) & 1, (h >> 8) & 15))
            share = {k: key.count(k) for k in set(key)}
            ml = [(S[1][i] - S[0][i]) / 100 for i in range(nb)]
            en = [(S[7][i] - t0) / 100 for i in range(nb)]
            for name, grp in (("xcc", lambda i: key[i][0]), ("blocks on the CU", lambda i: share[key[i]])):
                g = {}
                for i in range(nb):
                    g.setdefault(grp(i), []).append(i)
                print(f"N={N} by {name}: " + "  ".join(
                    f"{k}: n={len(v)} loop {q([ml[i] for i in v]):.1f}/{max(ml[i] for i in v):.1f} end "
                    f"{q([en[i] for i in v]):.1f}/{max(en[i] for i in v):.1f}" for k, v in sorted(g.items())))
            raw = os.environ.get("KT_RAW")
            if raw:  # per block: id, start, main-loop end, end (us from the first start), xcc, se, sh, cu
                with open(f"{raw}_{N}.csv", "w") as fh:
                    fh.write("block,start_us,loop_end_us,end_us,xcc,se,sh,cu,blocks_on_cu\n")
                    for i in range(nb):
                        fh.write(f"{i},{(S[0][i] - t0) / 100:.2f},{(S[1][i] - t0) / 100:.2f},{en[i]:.2f},"
                                 f"{key[i][0]},{key[i][1]},{key[i][2]},{key[i][3]},{share[key[i]]}\n")
            slow = sorted(range(nb), key=lambda i: -ml[i])[:12]
            print(f"N={N} slowest main loops (block: us xcc/se/sh/cu, blocks on the CU):",
                  " ".join(f"{i}:{ml[i]:.1f} {key[i][0]}/{key[i][1]}/{key[i][2]}/{key[i][3]},{share[key[i]]}" for i in slow))


if __name__ == "__main__":
    main()
