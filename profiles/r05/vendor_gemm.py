"""The vendor library's fp32 GEMM on the headline's two GEMM shapes, for scale: torch.matmul (hipBLASLt /
rocBLAS on ROCm) with TF32 off, i.e. the same exact-fp32 arithmetic class as the engine's v_mfma_f32_32x32x2_f32
kernels. Plain GEMMs only (no bias / ReLU / fused head / fold / split-K slabs), so they bound from below what an
unfused route would cost. Prints one JSON line per shape: median of 50 timed launches (HIP events)."""
import json
import torch

torch.backends.cuda.matmul.allow_tf32 = False
torch.backends.cudnn.allow_tf32 = False
PEAK = 157.3  # TFLOP/s, fp32 MFMA dense (MI355X_MICROARCH.md)


def timeit(fn, n=50):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    g = torch.Generator(device="cuda").manual_seed(1)
    for name, M, K, N, tA in [("forward X W (60000x784 @ 784x128)", 60000, 784, 128, False),
                              ("dW X^T delta (784x60000 @ 60000x128)", 784, 60000, 128, True),
                              ("forward, 8-rank shard (7500x784 @ 784x128)", 7500, 784, 128, False),
                              ("dW, 8-rank shard (784x7500 @ 7500x128)", 784, 7500, 128, True)]:
        if tA:
            A = torch.randn(K, M, device="cuda", generator=g).t()  # X^T as a transposed view of X [K][M]
        else:
            A = torch.randn(M, K, device="cuda", generator=g)
        B = torch.randn(K, N, device="cuda", generator=g)
        C = torch.empty(M, N, device="cuda")
        us = timeit(lambda: torch.matmul(A, B, out=C))
        tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
        print(json.dumps({"gemm": name, "us": round(us, 2), "tflops": round(tf, 2), "frac_fp32_peak": round(tf / PEAK, 4)}))


if __name__ == "__main__":
    main()
