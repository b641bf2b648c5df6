// Small-tile GEMM main-loop micro-benchmark (gfx950): the forward GEMM's row tile per shard size
// (32 / 64 / 128 x 128 at 7500 / 15000 / 30000 / 60000 rows of 784 -> 128: Mlp::plan's rule).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../lbfgs-ffnn_amd/csrc gemm_small.hip -o gemm_small
// Every variant runs the library's own gemm_glds_kernel (EPI_FWD epilogue: no head) on synthetic
// operands. Earlier revisions of this file (git history) also timed the PIPE / LDR / register-staged
// variants and operands with a zero row stride (L1/L2-resident): profiles/r02/gemm_small_tiles.txt.
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
  // forward GEMM tile per shard size (EPI_FWD, 784 -> 128): rows of a 1/2/4/8-rank shard of N = 60000
  for (long long M : {7500LL, 15000LL, 30000LL, 60000LL}) {
    GemmK k{};
    k.M = int(M);
    k.N = Out;
    k.K = In;
    k.k_chunk = In;
    k.A = X;
    k.lda = In;
    k.a_mvalid = int(M);
    k.a_ones = -1;
    k.a_vec = 1;
    k.B = W;
    k.ldb = Out;
    k.b_vec = 1;
    k.C = C;
    k.ldc = Out;
    k.act = ACT_RELU;
    const double fl = 2.0 * M * In * Out;
    char nm[96];
    snprintf(nm, sizeof nm, "fwd 32x128 KW2 NS4 M=%lld", M);
    run<1, 4, 1, 1, true, false, EPI_FWD, 4, 2, false>(nm, k, dim3(1, unsigned((M + 31) / 32), 1), reps, fl);
    snprintf(nm, sizeof nm, "fwd 64x128 NS3 M=%lld", M);
    run<2, 2, 1, 2, true, false, EPI_FWD, 3, 1, false>(nm, k, dim3(1, unsigned((M + 63) / 64), 1), reps, fl);
    snprintf(nm, sizeof nm, "fwd 64x128 KW2 NS3 M=%lld", M);
    run<2, 2, 1, 2, true, false, EPI_FWD, 3, 2, false>(nm, k, dim3(1, unsigned((M + 63) / 64), 1), reps, fl);
    snprintf(nm, sizeof nm, "fwd 128x128 NS2 M=%lld", M);
    run<2, 2, 2, 2, true, false, EPI_FWD, 2, 1, false>(nm, k, dim3(1, unsigned((M + 127) / 128), 1), reps, fl);
  }
  CK(hipDeviceSynchronize());
  return 0;
}
