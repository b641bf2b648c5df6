// Small-tile GEMM main-loop micro-benchmark (gfx950): what limits the 32 x 128 forward tile of a rank's
// 7500-row shard (one workgroup per CU) and the 64 x 64 split-K dW tile?
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../lbfgs-ffnn_amd/csrc gemm_small.hip -o gemm_small
// Every variant runs the library's own gemm_glds_kernel (EPI_FWD / EPI_STORE epilogue: no head) on
// synthetic operands; the "A0" / "B0" data modes give an operand a zero row stride, so all its k-tiles
// hit the same few cache lines (L1/L2 resident): what is left is the in-core cost of the loop.
#include "gemm.hip"

#include <cstdio>
#include <vector>

using namespace lbf;

#define CK(x)                                                                                                \
  do {                                                                                                       \
    hipError_t e = (x);                                                                                      \
    if (e != hipSuccess) {                                                                                   \
      printf("%s line %d\n", hipGetErrorString(e), __LINE__);                                                \
      return 1;                                                                                              \
    }                                                                                                        \
  } while (0)

template <int WM, int WN, int TM, int TN, bool AKC, bool BKC, int EPI, int NS, int KW, bool PIPE, bool LDR = false>
static float run(const char *name, GemmK k, dim3 grid, int reps, double flops) {
  const dim3 block(256 * KW);
  for (int i = 0; i < 10; ++i)
    hipLaunchKernelGGL((gemm_glds_kernel<WM, WN, TM, TN, AKC, BKC, EPI, false, NS, KW, PIPE, LDR>), grid, block, 0, 0, k);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((gemm_glds_kernel<WM, WN, TM, TN, AKC, BKC, EPI, false, NS, KW, PIPE, LDR>), grid, block, 0, 0, k);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1e3 / reps;
  const int nk = (k.k_chunk + 31) / 32;
  printf("%-34s grid %4u x %3u x %3u  %8.2f us/launch  %6.3f us/k-tile  %6.1f TF/s\n", name, grid.x, grid.y, grid.z,
         us, us / nk, flops / us / 1e6);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return float(us);
}

template <int WM, int WN, int TM, int TN, bool AKC, bool BKC, int EPI, int KW, int PF>
static float run_rs(const char *name, GemmK k, dim3 grid, int reps, double flops) {
  const dim3 block(256 * KW);
  for (int i = 0; i < 10; ++i)
    hipLaunchKernelGGL((gemm_kernel<WM, WN, TM, TN, AKC, BKC, EPI, false, KW, PF, true>), grid, block, 0, 0, k);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((gemm_kernel<WM, WN, TM, TN, AKC, BKC, EPI, false, KW, PF, true>), grid, block, 0, 0, k);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1e3 / reps;
  const int nk = (k.k_chunk + 31) / 32;
  printf("%-34s grid %4u x %3u x %3u  %8.2f us/launch  %6.3f us/k-tile  %6.1f TF/s\n", name, grid.x, grid.y, grid.z,
         us, us / nk, flops / us / 1e6);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return float(us);
}

int main() {
  const int In = 784, Out = 128;
  const long long Mbig = 60000;
  float *X, *W, *C, *D;
  CK(hipMalloc(&X, Mbig * In * 4));
  CK(hipMalloc(&W, (long long)In * Out * 4 + 4096));
  CK(hipMalloc(&C, Mbig * Out * 4 * 4));
  CK(hipMalloc(&D, Mbig * Out * 4));
  CK(hipMemset(X, 0, Mbig * In * 4));
  CK(hipMemset(W, 0, (long long)In * Out * 4 + 4096));
  CK(hipMemset(D, 0, Mbig * Out * 4));
  const int reps = 200;
  for (int mode = 0; mode < 3; mode += 2) { // 0: real operands, 1: A0 (X row stride 0), 2: B0 (W row stride 0)
    const char *mn = mode == 0 ? "" : (mode == 1 ? " A0" : " B0");
    for (long long M : {7500LL, 60000LL}) {
      GemmK k{};
      k.M = int(M);
      k.N = Out;
      k.K = In;
      k.k_chunk = In;
      k.A = X;
      k.lda = mode == 1 ? 0 : In;
      k.a_mvalid = int(M);
      k.a_ones = -1;
      k.a_vec = 1;
      k.B = W;
      k.ldb = mode == 2 ? 0 : Out;
      k.b_vec = 1;
      k.C = C;
      k.ldc = Out;
      k.act = ACT_RELU;
      const double fl = 2.0 * M * In * Out;
      char nm[96];
      if (M == 7500) {
        const dim3 g32(1, unsigned((M + 31) / 32), 1);
        snprintf(nm, sizeof nm, "fwd 32x128 KW2 NS4%s M=%lld", mn, M);
        run<1, 4, 1, 1, true, false, EPI_FWD, 4, 2, false>(nm, k, g32, reps, fl);
        snprintf(nm, sizeof nm, "fwd 32x128 KW1 NS4 PIPE%s M=%lld", mn, M);
        run<1, 4, 1, 1, true, false, EPI_FWD, 4, 1, true>(nm, k, g32, reps, fl);
        snprintf(nm, sizeof nm, "fwd 32x128 KW1 NS5 PIPE%s M=%lld", mn, M);
        run<1, 4, 1, 1, true, false, EPI_FWD, 5, 1, true>(nm, k, g32, reps, fl);
        snprintf(nm, sizeof nm, "fwd 32x128 KW1 NS4%s M=%lld", mn, M);
        run<1, 4, 1, 1, true, false, EPI_FWD, 4, 1, false>(nm, k, g32, reps, fl);
        snprintf(nm, sizeof nm, "fwd 32x128 LDR NS4%s M=%lld", mn, M);
        run<1, 4, 1, 1, true, false, EPI_FWD, 4, 2, false, true>(nm, k, g32, reps, fl);
        snprintf(nm, sizeof nm, "fwd 32x128 LDR NS6%s M=%lld", mn, M);
        run<1, 4, 1, 1, true, false, EPI_FWD, 6, 2, false, true>(nm, k, g32, reps, fl);
        snprintf(nm, sizeof nm, "fwd 32x128 RS KW1 PF2%s M=%lld", mn, M);
        run_rs<1, 4, 1, 1, true, false, EPI_FWD, 1, 2>(nm, k, g32, reps, fl);
        snprintf(nm, sizeof nm, "fwd 32x128 RS KW2 PF2%s M=%lld", mn, M);
        run_rs<1, 4, 1, 1, true, false, EPI_FWD, 2, 2>(nm, k, g32, reps, fl);
        snprintf(nm, sizeof nm, "fwd 32x128 RS KW1 PF3%s M=%lld", mn, M);
        run_rs<1, 4, 1, 1, true, false, EPI_FWD, 1, 3>(nm, k, g32, reps, fl);
      }
      const dim3 g128(1, unsigned((M + 127) / 128), 1);
      snprintf(nm, sizeof nm, "fwd 128x128 NS2%s M=%lld", mn, M);
      run<2, 2, 2, 2, true, false, EPI_FWD, 2, 1, false>(nm, k, g128, reps, fl);
      snprintf(nm, sizeof nm, "fwd 128x128 LDR NS2%s M=%lld", mn, M);
      run<2, 2, 2, 2, true, false, EPI_FWD, 2, 2, false, true>(nm, k, g128, reps, fl);
      snprintf(nm, sizeof nm, "fwd 128x128 RS PF2%s M=%lld", mn, M);
      run_rs<2, 2, 2, 2, true, false, EPI_FWD, 1, 2>(nm, k, g128, reps, fl);
    }
  }
  // dW of the shard: [768 x 128] = X^T delta over 7500 rows, 64 x 64 tiles, 20 splits of 384 rows
  for (int mode = 0; mode < 3; mode += 2) {
    const char *mn = mode == 0 ? "" : (mode == 1 ? " A0" : " B0");
    const int B = 7500, splits = 20, kc = 384;
    GemmK k{};
    k.M = 768;
    k.N = Out;
    k.K = B;
    k.k_chunk = kc;
    k.A = X;
    k.lda = mode == 1 ? 0 : In;
    k.a_mvalid = 768;
    k.a_ones = -1;
    k.a_vec = 1;
    k.B = D;
    k.ldb = mode == 2 ? 0 : Out;
    k.b_vec = 1;
    k.C = C;
    k.ldc = Out;
    k.slab_stride = 768LL * Out;
    const double fl = 2.0 * B * 768 * Out;
    char nm[96];
    snprintf(nm, sizeof nm, "dW 64x64 NS5 s20%s", mn);
    run<2, 2, 1, 1, false, false, EPI_STORE, 5, 1, false>(nm, k, dim3(2, 12, splits), reps, fl);
    snprintf(nm, sizeof nm, "dW 64x64 NS5 PIPE s20%s", mn);
    run<2, 2, 1, 1, false, false, EPI_STORE, 5, 1, true>(nm, k, dim3(2, 12, splits), reps, fl);
    k.k_chunk = 7500 / 10 / 32 * 32 + 32;
    snprintf(nm, sizeof nm, "dW 64x64 NS5 s10%s", mn);
    run<2, 2, 1, 1, false, false, EPI_STORE, 5, 1, false>(nm, k, dim3(2, 12, 10), reps, fl);
    snprintf(nm, sizeof nm, "dW 64x64 NS5 PIPE s10%s", mn);
    run<2, 2, 1, 1, false, false, EPI_STORE, 5, 1, true>(nm, k, dim3(2, 12, 10), reps, fl);
    snprintf(nm, sizeof nm, "dW 64x64 LDR NS5 s10%s", mn);
    run<2, 2, 1, 1, false, false, EPI_STORE, 5, 2, false, true>(nm, k, dim3(2, 12, 10), reps, fl);
    snprintf(nm, sizeof nm, "dW 64x64 RS PF2 s10%s", mn);
    run_rs<2, 2, 1, 1, false, false, EPI_STORE, 1, 2>(nm, k, dim3(2, 12, 10), reps, fl);
    k.k_chunk = kc;
    snprintf(nm, sizeof nm, "dW 64x64 RS PF2 s20%s", mn);
    run_rs<2, 2, 1, 1, false, false, EPI_STORE, 1, 2>(nm, k, dim3(2, 12, 20), reps, fl);
    k.k_chunk = 7500 / 10 / 32 * 32 + 32;
    k.k_chunk = kc;
    snprintf(nm, sizeof nm, "dW 128x128 NS2 s20%s", mn);
    run<2, 2, 2, 2, false, false, EPI_STORE, 2, 1, false>(nm, k, dim3(1, 6, splits), reps, fl);
    k.k_chunk = 7500 / 40 / 32 * 32 + 32;
    snprintf(nm, sizeof nm, "dW 128x128 NS2 s40%s", mn);
    run<2, 2, 2, 2, false, false, EPI_STORE, 2, 1, false>(nm, k, dim3(1, 6, unsigned((B + k.k_chunk - 1) / k.k_chunk)), reps, fl);
    snprintf(nm, sizeof nm, "dW 128x128 LDR NS3 s40%s", mn);
    run<2, 2, 2, 2, false, false, EPI_STORE, 3, 2, false, true>(nm, k, dim3(1, 6, unsigned((B + k.k_chunk - 1) / k.k_chunk)), reps, fl);
  }
  CK(hipDeviceSynchronize());
  return 0;
}
