// Where a 32 x 128 fp32 GEMM k-tile's time goes on gfx950 (round 5). The library's 32 x 128 forward tile runs
// 0.92 us per 32-deep k-tile (profiles/r02 gemm_small_tiles) against 0.49 us of MFMA issue (16
// v_mfma_f32_32x32x2_f32 per wave, 64 cycles each), and profiles/micro/delivery.hip shows the LDS-DMA path
// delivering 55-68 B/cycle/CU, five times what that loop moves. This kernel is the same loop skeleton (4 waves,
// one workgroup per CU, wave w owns output columns 32w..32w+31, BK = 32 k-tiles of A 32 x 32 and B 32 x 128
// staged by LDS-DMA into an NS-deep ring) with each ingredient switchable:
//   DMA  issue the 5 pieces per wave per k-tile (else the ring keeps stale bytes)
//   BAR  counted vmcnt + s_barrier per k-tile
//   RD   fragments read from LDS (else registers reused)
//   IL   the DMA pieces interleaved between the MFMAs (else issued in a burst after the barrier)
//   BK   32 or 64 (64: two MFMA groups per barrier)
// Reports us per launch (events), in-kernel cycles per k-tile (s_memtime, median block) and the in-kernel clock.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 loop32.hip -o loop32 && ./loop32
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#define CK(x)                                                                                                \
  do {                                                                                                       \
    hipError_t e = (x);                                                                                      \
    if (e != hipSuccess) {                                                                                   \
      printf("%s line %d\n", hipGetErrorString(e), __LINE__);                                                \
      return 1;                                                                                              \
    }                                                                                                        \
  } while (0)

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int K = 784, M = 7500, NCOL = 128;

template <int N> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// A: [M][K] row-major (k-contiguous rows), B: [K][NCOL] row-major. Out: [M][NCOL].
template <bool DMA, bool BAR, bool RD, bool IL, int BK, int NS>
__global__ __launch_bounds__(256) void loop_kernel(const float *A, const float *B, float *C, unsigned long long *stamps) {
  constexpr int STG = (32 + NCOL) * BK;       // floats per stage
  constexpr int PW = (32 + NCOL) * BK / 1024;  // 1-KiB pieces per wave per k-tile (4 waves x 256 floats)
  __shared__ __attribute__((aligned(16))) float lds[NS * STG];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int m0 = blockIdx.x * 32;
  const int nk = K / BK + (K % BK ? 1 : 0);
  // piece j = wave + 4 i of a k-tile: A pieces first (32 rows x BK = 32 BK floats: BK/8 pieces), then B
  constexpr int PA = 32 * BK / 256;
  unsigned long long src0[PW], step[PW];
  int dst[PW];
  // A image: k-contiguous rows of BK floats, 16-B chunk slot c of row r holds global chunk c ^ sw(r) (the
  // library's source-address swizzle: conflict-free ds_read_b128 fragment reads); B image: [BK][128] as is.
  auto sw = [](int r) { return BK == 32 ? ((r >> 1) & 7) : (r & 15); };
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int j = wave + 4 * i;
    if (j < PA) { // A piece: 256 floats = 256/BK rows of BK floats
      constexpr int CPR = BK / 4; // chunks per row
      const int r = j * (256 / BK) + lane / CPR, c = lane % CPR;
      const int row = min(m0 + r, M - 1);
      src0[i] = reinterpret_cast<unsigned long long>(A + (long long)row * K + 4 * (c ^ sw(r)));
      step[i] = BK * sizeof(float);
    } else { // B piece: 256 floats = 2 k-rows of 128
      const int jj = j - PA;
      const int kr = jj * 2 + (lane * 4) / NCOL, c = (lane * 4) % NCOL;
      src0[i] = reinterpret_cast<unsigned long long>(B + (long long)kr * NCOL + c);
      step[i] = (unsigned long long)BK * NCOL * sizeof(float);
    }
    dst[i] = j * 256;
  }
  auto piece = [&](int tt, int i) {
    const int kt = tt * BK;
    const unsigned long long a = src0[i] + (unsigned long long)tt * step[i];
    const bool ok = kt + (BK - 1) < K + BK; // (kept simple: K % 4 == 0, in-bounds reads past K are inside B / A)
    __builtin_amdgcn_global_load_lds((glb_void_t *)(ok ? a : src0[i]), (lds_void_t *)(lds + (tt % NS) * STG + dst[i]),
                                     16, 0, 0);
  };
  auto issue = [&](int tt) {
#pragma unroll
    for (int i = 0; i < PW; ++i) piece(tt, i);
  };
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float af[BK / 2], bf[BK / 2];
#pragma unroll
  for (int s = 0; s < BK / 2; ++s) {
    af[s] = 1.0f + 1e-3f * s;
    bf[s] = 1.0f - 1e-3f * s;
  }
  if (DMA)
    for (int tt = 0; tt < NS - 1 && tt < nk; ++tt) issue(tt);
  unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < nk; ++i) {
    if (BAR) {
      if (DMA) {
        if (i + NS - 2 < nk) vm_wait<PW * (NS - 2)>();
        else vm_wait<0>();
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    const bool more = DMA && i + NS - 1 < nk;
    if (more && !IL) issue(i + NS - 1);
    const float *As = lds + (i % NS) * STG, *Bs = As + 32 * BK;
    if (RD) { // lane half h consumes k = (BK/2) h + s at step s (the library's k permutation)
      constexpr int SQ = BK / 8; // quads per lane half
#pragma unroll
      for (int q = 0; q < SQ; ++q) {
        const float4 v = *reinterpret_cast<const float4 *>(As + li * BK + 4 * ((lh * SQ + q) ^ sw(li)));
        af[4 * q + 0] = v.x;
        af[4 * q + 1] = v.y;
        af[4 * q + 2] = v.z;
        af[4 * q + 3] = v.w;
      }
#pragma unroll
      for (int s = 0; s < BK / 2; ++s) bf[s] = Bs[(lh * (BK / 2) + s) * NCOL + wave * 32 + li];
    }
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) {
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bf[s], acc, 0, 0, 0);
      if (IL && more && s < PW) piece(i + NS - 1, s);
    }
  }
  unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (t == 0) {
    stamps[2 * blockIdx.x] = c1 - c0;
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + 8 * (r / 4) + lh * 4 + (r % 4), col = wave * 32 + li;
    if (row < M) C[(long long)row * NCOL + col] = acc[r];
  }
}

// The same 32 x 128 tile with NO LDS in the main loop: the four waves split each 32-deep k-tile (wave w
// takes k 8w .. 8w+7, lane half h the 4 consecutive k 8w+4h .. +3), so no operand is shared between waves:
// every lane loads its A quad X[row][k..k+3] and, per k, one 16-B quad of the W row (columns 4 li .. +3)
// straight into registers, PD k-tiles ahead. The quad's 4 columns feed 4 accumulators (column block cb holds
// columns 4 j + cb: a permutation of the output columns), 16 MFMAs per wave per k-tile from 4 independent
// chains; at the end the four waves' partial tiles are summed in wave order through LDS into the standard
// accumulator layout (wave w owns columns 32w .. 32w+31).
typedef float f32x4v __attribute__((ext_vector_type(4)));
template <int PD>
__global__ __launch_bounds__(256, 1) void direct_kernel(const float *A, const float *B, float *C,
                                                        unsigned long long *stamps, int kdim) {
  __shared__ __attribute__((aligned(16))) float red[4 * 16 * 2 * 128];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int m0 = blockIdx.x * 32;
  const int nk = (kdim + 31) / 32; // runtime, as in the library (no full unroll)
  const int row = min(m0 + li, M - 1);
  const int k4 = 8 * wave + 4 * lh;
  const float *ap = A + (long long)row * K + k4;
  const float *bp = B + (long long)k4 * NCOL + 4 * li;
  f32x16 acc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  f32x4v ra[PD], rb[PD][4];
  bool okm[PD];
  auto load = [&](int tt, int slot) { // clamped and unconditional; the mask is applied at the use
    const bool ok = tt * 32 + k4 < kdim;
    const long long ko = ok ? (long long)tt * 32 : 0;
    okm[slot] = ok;
    ra[slot] = *reinterpret_cast<const f32x4v *>(ap + ko);
#pragma unroll
    for (int s = 0; s < 4; ++s) rb[slot][s] = *reinterpret_cast<const f32x4v *>(bp + (ko + s) * NCOL);
  };
#pragma unroll
  for (int p = 0; p < PD; ++p) load(p, p);
  unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i0 = 0; i0 < nk; i0 += PD) {
#pragma unroll
    for (int p = 0; p < PD; ++p) {
      const int i = i0 + p;
      if (i < nk) { // wave-uniform
        f32x4v a = ra[p];
        if (!okm[p]) a = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], rb[p][s][c], acc[c], 0, 0, 0);
      }
      // the slot's next k-tile, issued after the MFMAs that read it (no register copy, so no wait for the
      // new data inside this iteration), PD - 1 k-tiles of MFMAs ahead of its use; clamped, unconditional
      __builtin_amdgcn_sched_barrier(0);
      load(i + PD, p);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // partial tiles summed in wave order into the standard layout
#pragma unroll
  for (int r = 0; r < 16; ++r)
    *reinterpret_cast<f32x4v *>(&red[((wave * 16 + r) * 2 + lh) * 128 + li * 4]) =
        f32x4v{acc[0][r], acc[1][r], acc[2][r], acc[3][r]};
  __syncthreads();
  f32x16 out;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) v += red[((w * 16 + r) * 2 + lh) * 128 + 32 * wave + li];
    out[r] = v;
  }
  unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (t == 0) {
    stamps[2 * blockIdx.x] = c1 - c0;
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int rr = m0 + 8 * (r / 4) + lh * 4 + (r % 4), col = wave * 32 + li;
    if (rr < M) C[(long long)rr * NCOL + col] = out[r];
  }
}

// Column split: wave w owns columns 32w .. 32w+31 over the WHOLE K (standard accumulator layout, no
// cross-wave reduction): per 8 k a lane loads one 16-B A quad X[row][k..k+3] (lane half h: k = 8j + 4h + s;
// the four waves read the same A bytes, L1 hits) and 4 W values W[k][32w + li] (dwords, 2 x 128 B per
// instruction); 4 MFMAs per 8 k on one accumulator chain.
template <int PD>
__global__ __launch_bounds__(256, 1) void colsplit_kernel(const float *A, const float *B, float *C,
                                                          unsigned long long *stamps, int kdim) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int m0 = blockIdx.x * 32;
  const int n8 = (kdim + 7) / 8;
  const int row = min(m0 + li, M - 1);
  const float *ap = A + (long long)row * K + 4 * lh;
  const float *bp = B + (long long)(4 * lh) * NCOL + 32 * wave + li;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  f32x4v ra[PD];
  float rb[PD][4];
  bool okm[PD];
  auto load = [&](int j, int slot) {
    const bool ok = 8 * j + 4 * lh < kdim;
    const long long ko = ok ? 8LL * j : 0;
    okm[slot] = ok;
    ra[slot] = *reinterpret_cast<const f32x4v *>(ap + ko);
#pragma unroll
    for (int s = 0; s < 4; ++s) rb[slot][s] = bp[(ko + s) * NCOL];
  };
#pragma unroll
  for (int p = 0; p < PD; ++p) load(p, p);
  unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int j0 = 0; j0 < n8; j0 += PD) {
#pragma unroll
    for (int p = 0; p < PD; ++p) {
      const int j = j0 + p;
      if (j < n8) {
        f32x4v a = ra[p];
        if (!okm[p]) a = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], rb[p][s], acc, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      load(j + PD, p);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (t == 0) {
    stamps[2 * blockIdx.x] = c1 - c0;
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int rr = m0 + 8 * (r / 4) + lh * 4 + (r % 4), col = wave * 32 + li;
    if (rr < M) C[(long long)rr * NCOL + col] = acc[r];
  }
}

// dW-shaped: C[m][n] = sum_k X[k][m] dZ[k][n] over a K chunk, a 128 x 128 output tile per workgroup (m 0..127 of
// the 784 input columns, all 128 n), wave w owns n-block w: per 2 k a lane loads the 16-B quad X[k][4 li .. +3]
// (lane half h: row k = 2j + h) feeding 4 m-blocks (m = 4 m' + r) and one dZ value dZ[k][32w + li]: 4 MFMAs on
// 4 accumulator chains per 2 k.
template <int PD>
__global__ __launch_bounds__(256, 1) void dw_direct_kernel(const float *X, const float *D, float *Cs, int kchunk,
                                                           unsigned long long *stamps) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int kb = blockIdx.x * kchunk;
  const int ke = min(M, kb + kchunk);
  const int n2 = (ke - kb + 1) / 2;
  const float *xp = X + (long long)(kb + lh) * K + 4 * li;
  const float *dp = D + (long long)(kb + lh) * NCOL + 32 * wave + li;
  f32x16 acc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  f32x4v rx[PD];
  float rd[PD];
  bool okm[PD];
  auto load = [&](int j, int slot) {
    const bool ok = kb + 2 * j + lh < ke;
    const long long ko = ok ? 2LL * j : 0;
    okm[slot] = ok;
    rx[slot] = *reinterpret_cast<const f32x4v *>(xp + ko * K);
    rd[slot] = dp[ko * NCOL];
  };
#pragma unroll
  for (int p = 0; p < PD; ++p) load(p, p);
  unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int j0 = 0; j0 < n2; j0 += PD) {
#pragma unroll
    for (int p = 0; p < PD; ++p) {
      const int j = j0 + p;
      if (j < n2) {
        const float d = okm[p] ? rd[p] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = __builtin_amdgcn_mfma_f32_32x32x2f32(rx[p][r], d, acc[r], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      load(j + PD, p);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (t == 0) {
    stamps[2 * blockIdx.x] = c1 - c0;
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
  float *cs = Cs + (long long)blockIdx.x * 128 * NCOL;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int mp = 8 * (e / 4) + lh * 4 + (e % 4);
      cs[(4 * mp + r) * NCOL + 32 * wave + li] = acc[r][e];
    }
}

template <class KF>
static int timed(const char *name, KF launch, unsigned long long *st, int nb, double cyc_div, const char *unit) {
  for (int i = 0; i < 20; ++i) launch();
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int reps = 200;
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  std::vector<unsigned long long> h(2 * nb);
  CK(hipMemcpy(h.data(), st, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  std::vector<double> cyc(nb), ghz(nb);
  for (int i = 0; i < nb; ++i) {
    cyc[i] = double(h[2 * i]);
    ghz[i] = double(h[2 * i]) / (double(h[2 * i + 1]) * 10.0);
  }
  std::sort(cyc.begin(), cyc.end());
  std::sort(ghz.begin(), ghz.end());
  printf("%-28s %7.2f us/launch  %7.1f cyc/%s (median block) at %.2f GHz\n", name, ms * 1e3 / reps,
         cyc[nb / 2] / cyc_div, unit, ghz[nb / 2]);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 0;
}

template <int PD>
static int run_direct(const char *name, const float *A, const float *B, float *C, unsigned long long *st, int nb) {
  auto k = direct_kernel<PD>;
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k, dim3(nb), dim3(256), 0, 0, A, B, C, st, K);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int reps = 200;
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, dim3(nb), dim3(256), 0, 0, A, B, C, st, K);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  std::vector<unsigned long long> h(2 * nb);
  CK(hipMemcpy(h.data(), st, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  std::vector<double> cyc(nb), ghz(nb);
  for (int i = 0; i < nb; ++i) {
    cyc[i] = double(h[2 * i]);
    ghz[i] = double(h[2 * i]) / (double(h[2 * i + 1]) * 10.0);
  }
  std::sort(cyc.begin(), cyc.end());
  std::sort(ghz.begin(), ghz.end());
  const int nk = (K + 31) / 32;
  printf("%-28s %7.2f us/launch  %7.1f cyc/k32 (median block)  %.3f us/k32 at %.2f GHz  MFMA floor %d cyc/k32\n", name,
         ms * 1e3 / reps, cyc[nb / 2] / nk, cyc[nb / 2] / nk / (ghz[nb / 2] * 1e3), ghz[nb / 2], 16 * 64);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 0;
}

template <bool DMA, bool BAR, bool RD, bool IL, int BK, int NS>
static int run(const char *name, const float *A, const float *B, float *C, unsigned long long *st, int nb) {
  auto k = loop_kernel<DMA, BAR, RD, IL, BK, NS>;
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k, dim3(nb), dim3(256), 0, 0, A, B, C, st);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int reps = 200;
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, dim3(nb), dim3(256), 0, 0, A, B, C, st);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  std::vector<unsigned long long> h(2 * nb);
  CK(hipMemcpy(h.data(), st, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  std::vector<double> cyc(nb), ghz(nb);
  for (int i = 0; i < nb; ++i) {
    cyc[i] = double(h[2 * i]);
    ghz[i] = double(h[2 * i]) / (double(h[2 * i + 1]) * 10.0); // memrealtime: 100 MHz
  }
  std::sort(cyc.begin(), cyc.end());
  std::sort(ghz.begin(), ghz.end());
  const int nk = K / BK + (K % BK ? 1 : 0);
  printf("%-28s %7.2f us/launch  %7.1f cyc/k32 (median block)  %.3f us/k32 at %.2f GHz  MFMA floor %d cyc/k32\n", name,
         ms * 1e3 / reps, cyc[nb / 2] / nk * 32.0 / BK, cyc[nb / 2] / nk * 32.0 / BK / (ghz[nb / 2] * 1e3),
         ghz[nb / 2], 16 * 64);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 0;
}

int main() {
  float *A, *B, *C;
  unsigned long long *st;
  const int nb = (M + 31) / 32;
  CK(hipMalloc(&A, size_t(M) * K * 4 + 65536));
  CK(hipMalloc(&B, size_t(K + 64) * NCOL * 4));
  CK(hipMalloc(&C, size_t(M) * NCOL * 4));
  CK(hipMalloc(&st, size_t(2 * nb) * 8));
  CK(hipMemset(A, 0, size_t(M) * K * 4 + 65536));
  CK(hipMemset(B, 0, size_t(K + 64) * NCOL * 4));
  printf("# 32 x 128 x %d fp32 tiles, %d workgroups (one per CU), 4 waves; k32 = one 32-deep k-step\n", K, nb);
  run<false, false, false, false, 32, 4>("mfma only", A, B, C, st, nb);
  run<false, false, true, false, 32, 4>("mfma + lds reads", A, B, C, st, nb);
  run<false, true, true, false, 32, 4>("+ barrier", A, B, C, st, nb);
  run<true, true, true, false, 32, 4>("+ dma burst (library)", A, B, C, st, nb);
  run<true, true, true, true, 32, 4>("+ dma interleaved", A, B, C, st, nb);
  run<true, true, true, false, 32, 3>("dma burst NS3", A, B, C, st, nb);
  run<true, true, true, false, 64, 3>("dma burst BK64 NS3", A, B, C, st, nb);
  run<true, true, true, true, 64, 3>("dma interleaved BK64 NS3", A, B, C, st, nb);
  run<false, true, true, false, 64, 3>("barrier, no dma BK64", A, B, C, st, nb);
  run<true, true, false, false, 32, 4>("dma burst, no lds reads", A, B, C, st, nb);
  // correctness of the direct form on random operands against a CPU fp64 reference (a few rows)
  {
    std::vector<float> ha(size_t(M) * K), hb(size_t(K + 64) * NCOL, 0.f), hc(size_t(M) * NCOL);
    unsigned x = 12345u;
    auto rnd = [&]() { x = x * 1664525u + 1013904223u; return float((x >> 8) & 0xffff) / 65536.0f - 0.5f; };
    for (auto &v : ha) v = rnd();
    for (int i = 0; i < K * NCOL; ++i) hb[i] = rnd();
    CK(hipMemcpy(A, ha.data(), ha.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
    run_direct<2>("direct PD2 (random)", A, B, C, st, nb);
    run_direct<3>("direct PD3 (random)", A, B, C, st, nb);
    run_direct<4>("direct PD4 (random)", A, B, C, st, nb);
    CK(hipMemcpy(hc.data(), C, hc.size() * 4, hipMemcpyDeviceToHost));
    auto check = [&](const char *what) {
      double worst = 0.0;
      for (int r : {0, 1, 31, 32, 4000, M - 1})
        for (int c = 0; c < NCOL; ++c) {
          double ref = 0.0, mag = 0.0;
          for (int k = 0; k < K; ++k) {
            ref += double(ha[size_t(r) * K + k]) * double(hb[size_t(k) * NCOL + c]);
            mag += std::fabs(double(ha[size_t(r) * K + k]) * double(hb[size_t(k) * NCOL + c]));
          }
          worst = std::max(worst, std::fabs(double(hc[size_t(r) * NCOL + c]) - ref) / mag);
        }
      printf("%s vs fp64: worst |d| / sum|a b| = %.3e\n", what, worst);
    };
    check("k-split direct");
    for (int pd : {2, 3, 4}) {
      char nm[64];
      snprintf(nm, sizeof nm, "colsplit PD%d (random)", pd);
      auto go = [&]() {
        if (pd == 2) hipLaunchKernelGGL(colsplit_kernel<2>, dim3(nb), dim3(256), 0, 0, A, B, C, st, K);
        if (pd == 3) hipLaunchKernelGGL(colsplit_kernel<3>, dim3(nb), dim3(256), 0, 0, A, B, C, st, K);
        if (pd == 4) hipLaunchKernelGGL(colsplit_kernel<4>, dim3(nb), dim3(256), 0, 0, A, B, C, st, K);
      };
      timed(nm, go, st, nb, (K + 31) / 32, "k32");
    }
    CK(hipMemcpy(hc.data(), C, hc.size() * 4, hipMemcpyDeviceToHost));
    check("colsplit direct");
    // dW shape: X [7500][784] (A above) and dZ [7500][128] (the first 7500 rows of B's buffer reused as random
    // data), 6 row tiles of 128 x 128 would each take a K chunk; here one m-tile (m 0..127), chunks of kc rows
    {
      float *D = nullptr, *Cs = nullptr;
      CK(hipMalloc(&D, size_t(M) * NCOL * 4 + 4096));
      std::vector<float> hd(size_t(M) * NCOL);
      for (auto &v : hd) v = rnd();
      CK(hipMemcpy(D, hd.data(), hd.size() * 4, hipMemcpyHostToDevice));
      for (int kc : {128, 192, 256}) {
        const int nbk = (M + kc - 1) / kc;
        CK(hipMalloc(&Cs, size_t(nbk) * 128 * NCOL * 4));
        char nm[64];
        snprintf(nm, sizeof nm, "dW direct kc%d PD4", kc);
        auto go = [&]() { hipLaunchKernelGGL(dw_direct_kernel<4>, dim3(nbk), dim3(256), 0, 0, A, D, Cs, kc, st); };
        timed(nm, go, st, nbk, kc / 32.0, "k32");
        std::vector<float> hs(size_t(nbk) * 128 * NCOL);
        CK(hipMemcpy(hs.data(), Cs, hs.size() * 4, hipMemcpyDeviceToHost));
        double worst = 0.0;
        for (int blk : {0, nbk - 1})
          for (int m : {0, 1, 5, 127})
            for (int n : {0, 33, 127}) {
              double ref = 0.0, mag = 0.0;
              for (int k = blk * kc; k < std::min(M, (blk + 1) * kc); ++k) {
                ref += double(ha[size_t(k) * K + m]) * double(hd[size_t(k) * NCOL + n]);
                mag += std::fabs(double(ha[size_t(k) * K + m]) * double(hd[size_t(k) * NCOL + n]));
              }
              worst = std::max(worst, std::fabs(double(hs[(size_t(blk) * 128 + m) * NCOL + n]) - ref) / mag);
            }
        printf("dW direct kc%d vs fp64: worst %.3e  (MFMA floor %d cyc per k32 of a 128 x 128 tile)\n", kc, worst,
               64 * 64);
        CK(hipFree(Cs));
      }
      CK(hipFree(D));
    }
    double worst = 0.0;
    for (int r : {0, 1, 31, 32, 4000, M - 1})
      for (int c = 0; c < NCOL; ++c) {
        double ref = 0.0, mag = 0.0;
        for (int k = 0; k < K; ++k) {
          ref += double(ha[size_t(r) * K + k]) * double(hb[size_t(k) * NCOL + c]);
          mag += std::fabs(double(ha[size_t(r) * K + k]) * double(hb[size_t(k) * NCOL + c]));
        }
        worst = std::max(worst, std::fabs(double(hc[size_t(r) * NCOL + c]) - ref) / mag);
      }
    printf("direct form vs fp64: worst |d| / sum|a b| = %.3e (fp32: ~1e-7)\n", worst);
    run<true, true, true, false, 32, 4>("library form (random)", A, B, C, st, nb);
  }
  CK(hipDeviceSynchronize());
  printf("loop32 ok\n");
  return 0;
}
