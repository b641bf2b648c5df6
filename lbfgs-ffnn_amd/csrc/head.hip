// Fused output layer ("head") for a small output width (Out <= 16) on a hidden width H <= 256.
//
// Each workgroup (4 waves) walks a fixed list of 64-sample tiles; from one LDS copy of a tile's
// activations A[b][0..H) it runs all three small products of the last layer on MFMA
// (v_mfma_f32_16x16x4_f32, Out padded to 16):
//   forward  Z = A W + b ; a = act(Z) ; d = a - y ; sse += d^2 ; dZ = d * act'(a) * inv_scale
//   delta    D = (dZ W^T) .* act_prev'(A)                        -> global, feeds the next dW GEMM
//   weights  [dW ; db] += [A | 1]^T dZ                             (accumulators stay in registers)
// and writes one [dW ; db] partial slab per workgroup at the end (reduced in fixed order afterwards:
// deterministic, no float atomics).
// Replaces for the last layer the reference's forward Sgemm + add_bias + activation, diff_kernel +
// Sdot + Sscal, activation_deriv + dW Sgemm + sum_rows + dX Sgemm (src/cuda/layer.cuh:48-105,
// src/cuda/network.cuh:97-119, src/cuda/kernels.cuh:74-153).
//
// 16x16x4 f32 MFMA: lane l feeds A[l&15][k = l>>4] and B[k = l>>4][l&15]; accumulator r of lane l is
// C[(l>>4)*4 + r][l&15]. Within a K-run of 4S values, lane group g = l>>4 consumes k = g*S + s at
// step s (a permutation of the summation order), so k-contiguous operands are ds_read_b128 runs.
#include "internal.hpp"
#include "head_core.hpp"
#include "kernels.hpp"
#include "wave.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>

namespace lbf {

__host__ __device__ int head_hsplit(long long B, int H);

namespace {

using namespace headc;

constexpr int MAX_WG = 512; // 2 workgroups per CU

// One tile's activations, A[b0 .. b0+TB)[0 .. H), in registers: every load issued before the first use
// from a clamped address and masked only when staged (a value masked at the load compiles to a branch
// around the load and a wait inside it: one round trip per 16-B chunk), so staging a tile is one memory
// round trip. H % 4 == 0 and 16-B aligned rows (vec); else the scalar path.
struct TileRegs {
  static constexpr int QPT = TB * (HMAX / 4) / 256; // 16-B chunks per thread (16 at H = 256)
  f32x4 v[QPT];
  int rows = 0;
  __device__ inline void load(const float *A, int H, int Hp, long long b0, int rows_) {
    const int t = threadIdx.x, Hq = H >> 2, hq = Hp >> 2;
    rows = rows_;
#pragma unroll
    for (int j = 0; j < QPT; ++j) {
      const int e = t + j * 256;
      const int r = e / hq, c4 = e - r * hq;
      const bool ok = e < TB * hq && r < rows_ && c4 < Hq;
      v[j] = *reinterpret_cast<const f32x4 *>(A + (ok ? (b0 + r) * H + 4 * c4 : 0LL));
    }
  }
  __device__ inline void store(const Smem &sm) const {
    const int t = threadIdx.x, hq = sm.Hp >> 2, Hq = sm.H >> 2;
#pragma unroll
    for (int j = 0; j < QPT; ++j) {
      const int e = t + j * 256;
      const int r = e / hq, c4 = e - r * hq;
      const bool ok = r < rows && c4 < Hq;
      if (e < TB * hq) *reinterpret_cast<f32x4 *>(sm.As + r * sm.LDA + 4 * c4) = ok ? v[j] : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
  }
};

// W (H x Out, <= 4096 values) in registers, loaded with the first tile: one round trip for both.
struct WRegs {
  static constexpr int PT = HMAX * HMAX_OUT / 256;
  float w[PT];
  float bias;
  __device__ inline void load(const float *P, int H, int Out) {
    const int t = threadIdx.x, n = H * Out;
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      const int e = t + j * 256;
      w[j] = P[e < n ? e : 0];
    }
    bias = P[(long long)H * Out + (t < Out ? t : 0)];
  }
  // Wt [16][LDA] and Wr [Hp][16], zeros outside Out x H (the caller zeroed both and barriered)
  __device__ inline void store(const Smem &s, int Out) const {
    const int t = threadIdx.x, n = s.H * Out;
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      const int e = t + j * 256;
      if (e < n) {
        const int i = e / Out, o = e - i * Out;
        s.Wt[o * s.LDA + i] = w[j];
        s.Wr[i * 16 + ocol(o)] = w[j];
      }
    }
    if (t < HMAX_OUT) s.bias[t] = t < Out ? bias : 0.0f;
  }
};

template <int QM>
__global__ __launch_bounds__(256) void head_kernel(const float *A, int H, const float *P, int Out, const float *Y,
                                                   const int *idx, long long B, int act_out, int act_prev,
                                                   double inv_scale, float *delta, float *slab, double *sse_part,
                                                   const int *abort) {
  if (abort && *abort) return;
  KT(30);
  extern __shared__ __attribute__((aligned(16))) float sh[];
  const Smem sm = carve(sh, H);
  const int t = threadIdx.x, LDA = sm.LDA, Hp = sm.Hp;
  const long long ntiles = (B + TB - 1) / TB;
  const bool vec = (H & 3) == 0 && ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(delta)) & 15) == 0;
  // H split over hsplit workgroups per tile group (few tiles): split hs covers 64 columns of delta and the
  // matching [dW ; db] row strips (the last one also the bias row)
  const int hsplit = head_hsplit(B, H), hs = int(blockIdx.x) % hsplit;
  const int nwt = int(gridDim.x) / hsplit; // workgroups along the tiles
  HRange hr;
  if (hsplit > 1) {
    hr.st0 = 4 * hs;
    hr.st1 = hs == hsplit - 1 ? (H + 1 + 15) / 16 : 4 * hs + 4;
    hr.cb0 = 4 * hs;
    hr.cb1 = 4 * hs + 4;
  }
  TileRegs tr;
  long long tl = int(blockIdx.x) / hsplit;
  if (vec) {
    // W first, then the first tile (64 KB per workgroup), both in flight during stage_w's zero fill; the
    // barrier orders LDS only, so staging W waits for W's loads alone (vmcnt counts in issue order), not
    // for the tile's (phase stamps, profiles/r03b/head/head_phases_*.txt: W staged 4.8 us after entry)
    WRegs wr;
    wr.load(P, H, Out);
    if (tl < ntiles) tr.load(A, H, Hp, tl * TB, int(min((long long)TB, B - tl * TB)));
    for (int e = t; e < 16 * LDA; e += 256) sm.Wt[e] = 0.0f;
    for (int e = t; e < Hp * 16; e += 256) sm.Wr[e] = 0.0f;
    lds_barrier();
    wr.store(sm, Out);
  } else {
    stage_w(sm, P, Out);
  }
  KT(31);
  f32x4 cw[QM];
#pragma unroll
  for (int q = 0; q < QM; ++q) cw[q] = (f32x4){0.f, 0.f, 0.f, 0.f};
  double sse = 0.0;
  TileArgs ta;
  ta.Y = Y;
  ta.idx = idx;
  ta.ys = nullptr;
  ta.Out = Out;
  ta.act_out = act_out;
  ta.act_prev = act_prev;
  ta.sc = float(inv_scale);
  ta.delta = delta;
  ta.vec = vec;
  ta.xr = nullptr;
  ta.nfold = 0;
  FoldAcc fa; // unused (no fold in the standalone kernel)
  for (; tl < ntiles; tl += nwt) {
    const long long b0 = tl * TB;
    const int rows = int(min((long long)TB, B - b0));
    // ---- stage the activation tile (prefetched in registers on the vector path) ----
    if (vec) {
      tr.store(sm);
      if (tl + nwt < ntiles) { // the block's next tile, in flight during this one's products
        const long long nb0 = (tl + nwt) * TB;
        tr.load(A, H, Hp, nb0, int(min((long long)TB, B - nb0)));
      }
    } else {
      for (int e = t; e < TB * Hp; e += 256) {
        const int r = e / Hp, c = e - r * Hp;
        sm.As[r * LDA + c] = (r < rows && c < H) ? A[(b0 + r) * H + c] : 0.0f;
      }
    }
    // LDS only: the next tile's prefetch (vector path) stays in flight through this tile's products
    if (vec) lds_barrier();
    else __syncthreads();
    KT(32);
    tile<false, QM, false>(sm, ta, b0, rows, cw, sse, fa, hr);
  }
  if (hs != 0) sse = 0.0; // every split computed the same loss; the first one reports it
  write_partials(sm, Out, cw, sse, slab + (long long)blockIdx.x * (H + 1) * Out, sse_part + blockIdx.x, hr);
  KT(33);
}

// Row head (RowHeadArgs): wave w of the block takes rows (4 blockIdx + w) rpw + r; lane l owns hidden
// columns l + 64 j, j < NJ; OP = Out rounded up to 4 (register arrays sized by it). Per row: the target row
// (through idx) and every slab value of the row's activations are requested before the first use (one
// round trip; rounds of 8 splits beyond that), then the activations in fwd_reduce_act's arithmetic (slabs
// summed in split order, fp32), Z = a W + b reduced across the wave in fp64 (DPP), the loss and dZ (every
// lane holds the row's dZ), delta = (dZ W^T) .* act_prev'(a) stored, and the row's [a | 1]^T dZ added into
// the wave's LDS partial (fp32, row order: what a register accumulator would hold); at the end the four
// waves' partials are summed in wave order into the block's slab.
template <int NJ, int OP>
__global__ __launch_bounds__(256) void rowhead_kernel(const RowHeadArgs a) {
  if (a.abort && *a.abort) return;
  KT(40);
  // [4][(H + 1) * Out] the waves' partials | [(H + 1) * Out] the output layer's W and bias
  extern __shared__ __attribute__((aligned(16))) float red[];
  __shared__ double ssew[4];
  constexpr int SU = 8;                                  // splits per column in flight per round
  constexpr int WST = ((64 * NJ + 1) * OP + 255) / 256; // staging loads of [W ; b] per thread
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int H = a.H, Out = a.Out, per = (H + 1) * Out;
  const long long rbase = ((long long)blockIdx.x * 4 + wave) * a.rpw;
  float *wl = red + 4 * per;
  // The output layer's [W ; b] (contiguous, (H + 1) Out floats) through LDS: the block reads it with
  // lane-contiguous loads; read per lane (its columns' rows of W, Out apart) the same values were 48
  // strided load instructions per wave, each touching ~40 cache lines. Every load below is unconditional
  // from a clamped address, NOT masked (a masked load compiles to a branch around it and a wait inside,
  // one round trip per value); clamped entries only ever meet zeros (av = 0 on columns past H, dZ = 0 on
  // outputs past Out) and those products are never stored.
  float wst[WST];
#pragma unroll
  for (int u = 0; u < WST; ++u) {
    const int e = t + 256 * u;
    wst[u] = a.P[e < per ? e : per - 1];
  }
  float hb[NJ];
  bool cv[NJ];
  int ccj[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = lane + 64 * j;
    cv[j] = c < H;
    ccj[j] = cv[j] ? c : H - 1;
    hb[j] = a.hbias[ccj[j]];
  }
  // the wave's first row (clamped into the batch): its target and slab values in the same round trip
  const bool pre = a.splits <= SU; // wave-uniform
  float ypre[OP], vpre[NJ][SU];
  {
    const long long b = rbase < a.B ? rbase : a.B - 1;
    const long long yrow = a.idx ? (long long)a.idx[b] : b;
#pragma unroll
    for (int o = 0; o < OP; ++o) ypre[o] = a.Y[yrow * Out + (o < Out ? o : Out - 1)];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const float *src = a.fslab + b * H + ccj[j];
#pragma unroll
      for (int u = 0; u < SU; ++u) vpre[j][u] = src[(long long)min(u, a.splits - 1) * a.stride];
    }
  }
  asm volatile("" ::: "memory");
  KT(41);
#pragma unroll
  for (int u = 0; u < WST; ++u) {
    const int e = t + 256 * u;
    if (e < per) wl[e] = wst[u];
  }
  lds_barrier();
  KT(42);
  float w2[NJ][OP], b2[OP], dbacc[OP];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int o = 0; o < OP; ++o) w2[j][o] = wl[ccj[j] * Out + (o < Out ? o : Out - 1)];
#pragma unroll
  for (int o = 0; o < OP; ++o) {
    b2[o] = wl[H * Out + (o < Out ? o : Out - 1)];
    dbacc[o] = 0.0f;
  }
  float *mine = red + wave * per;
  double sse = 0.0;
  int r = 0;
  for (; r < a.rpw; ++r) {
    const long long b = rbase + r;
    if (b >= a.B) break; // wave-uniform
    float yv[OP];
    float sum[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) sum[j] = 0.0f;
    if (r == 0 && pre) { // loaded above
#pragma unroll
      for (int o = 0; o < OP; ++o) yv[o] = ypre[o];
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int u = 0; u < SU; ++u)
          if (u < a.splits) sum[j] += vpre[j][u];
    } else {
      // ---- loads: the target row first (two deep through idx), then the slabs ----
      const long long yrow = a.idx ? (long long)a.idx[b] : b;
#pragma unroll
      for (int o = 0; o < OP; ++o) yv[o] = a.Y[yrow * Out + (o < Out ? o : Out - 1)];
      for (int k0 = 0; k0 < a.splits; k0 += SU) {
        float v[NJ][SU];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const float *src = a.fslab + b * H + ccj[j];
#pragma unroll
          for (int u = 0; u < SU; ++u) v[j][u] = src[(long long)min(k0 + u, a.splits - 1) * a.stride];
        }
        // every load of the round (and the targets) issued before the first use: the compiler may not sink
        // a load into the uniform branches below
        asm volatile("" ::: "memory");
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int u = 0; u < SU; ++u)
            if (k0 + u < a.splits) sum[j] += v[j][u];
      }
    }
    KT(43);
    // ---- activations (fwd_reduce_act's arithmetic) ----
    float av[NJ];
    with_act(a.act_prev, [&](auto AC) __attribute__((always_inline)) {
      constexpr int A = decltype(AC)::value;
#pragma unroll
      for (int j = 0; j < NJ; ++j) av[j] = cv[j] ? act_c<A>(sum[j] + hb[j]) : 0.0f;
    });
    // ---- Z = a W + b (fp64 partials, fixed DPP tree), loss, dZ: identical on every lane ----
    float dz[OP];
    with_act(a.act_out, [&](auto AC) __attribute__((always_inline)) {
      constexpr int A = decltype(AC)::value;
#pragma unroll
      for (int o = 0; o < OP; ++o) {
        dz[o] = 0.0f;
        if (o < Out) { // uniform
          double zp = 0.0;
#pragma unroll
          for (int j = 0; j < NJ; ++j) zp += double(av[j]) * double(w2[j][o]);
          const float z = float(wave_sum_f64(zp));
          const float outv = act_c<A>(z + b2[o]);
          const float d = outv - yv[o];
          sse += double(d) * double(d);
          dz[o] = d * dact_c<A>(outv) * float(a.inv_scale);
        }
      }
    });
    KT(44);
    // ---- delta = (dZ W^T) .* act_prev'(a), [dW ; db] += [a | 1]^T dZ ----
    with_act(a.act_prev, [&](auto AC) __attribute__((always_inline)) {
      constexpr int A = decltype(AC)::value;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        float dd = 0.0f;
#pragma unroll
        for (int o = 0; o < OP; ++o) dd += dz[o] * w2[j][o];
        if (cv[j]) a.delta[b * H + lane + 64 * j] = dd * dact_c<A>(av[j]);
      }
    });
    // the row's [a | 1]^T dZ into the wave's LDS partial: the first row stores (a wave-uniform branch, so no
    // LDS read is speculated and waited for per element, as the select form compiled to), later rows add
    if (r == 0) {
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        if (cv[j]) {
          float *row = mine + (lane + 64 * j) * Out;
#pragma unroll
          for (int o = 0; o < OP; ++o)
            if (o < Out) row[o] = av[j] * dz[o];
        }
    } else {
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        if (cv[j]) {
          float *row = mine + (lane + 64 * j) * Out;
#pragma unroll
          for (int o = 0; o < OP; ++o)
            if (o < Out) row[o] = row[o] + av[j] * dz[o];
        }
    }
#pragma unroll
    for (int o = 0; o < OP; ++o) dbacc[o] += dz[o];
  }
  if (r == 0) // a wave past the last row: zero partials
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      if (cv[j])
#pragma unroll
        for (int o = 0; o < OP; ++o)
          if (o < Out) mine[(lane + 64 * j) * Out + o] = 0.0f;
  KT(45);
  // ---- the block's slab: the four waves' partials summed in wave order ----
  if (lane == 0) {
#pragma unroll
    for (int o = 0; o < OP; ++o)
      if (o < Out) mine[H * Out + o] = dbacc[o];
    ssew[wave] = sse; // every lane holds the same sum
  }
  lds_barrier();
  KT(46);
  float *slab = a.slab + (long long)blockIdx.x * per;
  for (int e = t; e < per; e += 256) slab[e] = ((red[e] + red[per + e]) + red[2 * per + e]) + red[3 * per + e];
  if (t == 0) a.sse_part[blockIdx.x] = ((ssew[0] + ssew[1]) + ssew[2]) + ssew[3];
  KT(47);
}

} // namespace

bool rowhead_supported(int H, int Out) { return H >= 1 && H <= HMAX && Out >= 1 && Out <= HMAX_OUT; }
// rows per wave: one while the grid stays within 256 workgroups, then enough that it does (bounded slabs)
int rowhead_rpw(long long B) { return int(std::max(1LL, cdiv(std::max(1LL, B), 4LL * 256))); }
int rowhead_nwg(long long B) { return int(cdiv(std::max(1LL, B), 4LL * rowhead_rpw(B))); }

void rowhead(hipStream_t s, const RowHeadArgs &a) {
  LBF_REQUIRE(rowhead_supported(a.H, a.Out) && a.splits >= 1 && a.rpw == rowhead_rpw(a.B), "rowhead: shape");
  const size_t shmem = size_t(5) * (a.H + 1) * a.Out * sizeof(float); // 4 wave partials + [W ; b]
  const int nj = (a.H + 63) / 64, op = (a.Out + 3) / 4 * 4;
  const dim3 grid(unsigned(rowhead_nwg(a.B))), block(256);
  // <NJ, OP> for hidden widths up to 256 and outputs up to 16; the attribute once per instance (thread-safe)
#define LBF_ROWHEAD_CASE(NJ, OP)                                                                              \
  if (nj == NJ && op == OP) {                                                                                \
    static const bool attr_set = [] {                                                                        \
      LBF_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(rowhead_kernel<NJ, OP>),                    \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));                   \
      return true;                                                                                           \
    }();                                                                                                     \
    (void)attr_set;                                                                                          \
    hipLaunchKernelGGL((rowhead_kernel<NJ, OP>), grid, block, shmem, s, a);                                  \
    LBF_KERNEL_CHECK();                                                                                      \
    return;                                                                                                  \
  }
#define LBF_ROWHEAD_NJ(NJ) LBF_ROWHEAD_CASE(NJ, 4) LBF_ROWHEAD_CASE(NJ, 8) LBF_ROWHEAD_CASE(NJ, 12) LBF_ROWHEAD_CASE(NJ, 16)
  LBF_ROWHEAD_NJ(1)
  LBF_ROWHEAD_NJ(2)
  LBF_ROWHEAD_NJ(3)
  LBF_ROWHEAD_NJ(4)
#undef LBF_ROWHEAD_NJ
#undef LBF_ROWHEAD_CASE
  throw Error(2, "rowhead: no instance for this shape");
}

bool head_supported(int H, int Out) { return Out >= 1 && Out <= HMAX_OUT && H >= 1 && H <= HMAX; }
int head_tile(int) { return TB; }
// H splits per tile: 64 hidden columns per workgroup while a batch has at most 64 tiles (an S-LBFGS
// minibatch of 256 rows is 4 tiles: 4 workgroups on a 256-wide layer were 23 us, one CU each)
__host__ __device__ int head_hsplit(long long B, int H) {
  const long long nt = ((B > 1 ? B : 1) + TB - 1) / TB;
  const int hp = (H + 63) / 64;
  return nt <= 64 && hp > 1 ? hp : 1;
}
// Workgroups (== partial slabs): one per tile (x the H splits) up to MAX_WG, then a balanced number of
// tiles each.
int head_nwg(long long B, int H) {
  const long long nt = cdiv(std::max(1LL, B), TB);
  if (nt <= MAX_WG) return int(nt) * head_hsplit(B, H);
  const long long per = cdiv(nt, MAX_WG);
  return int(cdiv(nt, per));
}

void head_fused(hipStream_t s, const float *A, int H, const float *P, int Out, const float *Y, const int *idx,
                long long B, int act_out, int act_prev, double inv_scale, float *delta, float *slab,
                double *sse_part, const int *abort) {
  const size_t shmem = size_t(smem_floats(H)) * sizeof(float);
  // once per process, thread-safe (rank threads of an in-process group launch concurrently)
  static const bool attr_set = [] {
    const void *fns[] = {reinterpret_cast<const void *>(head_kernel<1>), reinterpret_cast<const void *>(head_kernel<2>),
                         reinterpret_cast<const void *>(head_kernel<3>), reinterpret_cast<const void *>(head_kernel<4>),
                         reinterpret_cast<const void *>(head_kernel<5>)};
    for (const void *f : fns)
      LBF_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 2048));
    return true;
  }();
  (void)attr_set;
  const dim3 grid(head_nwg(B, H)), block(256);
#define LBF_HEAD_LAUNCH(Q)                                                                                    \
  hipLaunchKernelGGL(head_kernel<Q>, grid, block, shmem, s, A, H, P, Out, Y, idx, B, act_out, act_prev, inv_scale, \
                     delta, slab, sse_part, abort)
  switch (qstrips(H)) {
  case 1: LBF_HEAD_LAUNCH(1); break;
  case 2: LBF_HEAD_LAUNCH(2); break;
  case 3: LBF_HEAD_LAUNCH(3); break;
  case 4: LBF_HEAD_LAUNCH(4); break;
  default: LBF_HEAD_LAUNCH(5); break;
  }
#undef LBF_HEAD_LAUNCH
  LBF_KERNEL_CHECK();
}

} // namespace lbf

#ifdef LBF_KTRACE
extern "C" int lbf_dbg_ktrace_head(unsigned long long *host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(lbf::lbf_kt_buf), size_t(n) * 8) == hipSuccess ? 0 : 1;
}
#endif
