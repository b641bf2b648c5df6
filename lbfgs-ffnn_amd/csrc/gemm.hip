// fp32 MFMA GEMM for the FFNN layers (gfx950, wave64).
//
// Replaces the reference's three cublasSgemm calls per layer (src/cuda/layer.cuh:51-103) and the
// add_bias / activation / activation_deriv kernels (src/cuda/kernels.cuh:74-133), which are fused
// into the epilogues here:
//   forward   Z = X * W + b, A = act(Z)            a_kc (X rows),  b mn-contiguous (W is [In][Out])
//   dX        D = (dZ * W^T) .* act'(A_prev)        a_kc (dZ rows), b_kc (W rows)
//   dW | db   [dW ; db] = [A_prev | 1]^T * dZ       both mn-contiguous, split-K over the batch
//
// MFMA: v_mfma_f32_32x32x2_f32 (exact f32 fma chain). Lane l feeds A[i = l&31][k = l>>5] and
// B[k = l>>5][j = l&31]; accumulator register r of lane l is C[(r&3) + 8*(r>>2) + 4*(l>>5)][l&31].
// The k index inside a 32-deep LDS tile is permuted so lane half h always consumes k = 16h + s at
// step s: a k-contiguous operand is then 16 consecutive floats per lane (4 x ds_read_b128) and an
// mn-contiguous operand is one conflict-free ds_read_b32 per step.
// Workgroup: 256 threads = 4 waves in a WM x WN grid, each wave TM x TN tiles of 32x32.
#include "act.hpp"
#include "head_core.hpp"
#include "internal.hpp"
#include "kernels.hpp"
#include "ls_rule.hpp"

#include <hip/hip_runtime.h>

#include <cstdlib>

namespace lbf {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct GemmK {
  int M, N, K, k_chunk;
  const float *A;
  long long lda;
  const int *a_idx;
  int a_mvalid, a_ones, a_vec;
  const float *B;
  long long ldb;
  int b_vec;
  float *C;
  long long ldc, slab_stride;
  const float *bias;
  int act;
  const float *aux;
  long long ldaux;
  int aux_act;
  const int *abort;
  int side_planes; // blockIdx.z < side_planes: side job (dispatched first); GEMM split = z - side_planes
  const float *side_slab;
  int side_splits;
  long long side_stride, side_count;
  float *side_dst;
  const float *head_P;
  int head_out, head_act;
  const float *head_Y;
  const int *head_idx;
  double head_inv_scale;
  float *head_delta, *head_slab;
  double *head_sse;
  int head_fold, head_fold_c0;
  const float *a_slab;
  int a_splits;
  long long a_slab_stride;
  const float *a_bias;
  int a_act;
  float *a_out;
  int gx, gy;   // this problem's tile grid (the grouped launch's grid is the larger of two)
  int group_z;  // grouped launch: GEMM planes of the first problem (the second's follow)
  int xcd_swz;  // split-K: deal each split's tiles to one XCD (xcd_tile below)
  EarlyLs early; // sse_part non-null: the speculative trial's Armijo test first (gemm_early_exit)
};

// EarlyLs (kernels.hpp): a speculative trial's sufficient-decrease test ahead of its backward. Threads 0..255
// sum the forward's SSE partials in tail_fin_body's order (thread t: r = t, t + 256, ..; wave sums;
// ((v0 + v1) + v2) + v3) and thread 0 applies ls_rule.hpp's test, so every block and the tail decide alike. The
// abort flag is read by thread 0 in the same round trip and the block's verdict goes through LDS: block 0 of
// this launch raises the flag while other blocks may be reading it, and one reader per block keeps the exit
// uniform. Block 0 publishes a failure as tail_fin_body publishes a rejection (status block words, abort flag,
// then the host record, its sequence word last). Runs before the kernel's first use of lds.
__device__ __forceinline__ bool gemm_early_exit(const GemmK &g, float *lds) {
  const EarlyLs &e = g.early;
  const int t = threadIdx.x;
  double *red = reinterpret_cast<double *>(lds);
  double sse = 0.0;
  if (t < 256)
    for (int r = t; r < e.nsse; r += 256) sse += e.sse_part[r];
  double gfo = 0.0, fold = 0.0, alpha0 = 0.0, accept_prev = 0.0;
  int abf = 0;
  if (t == 0) {
    const double *sc = e.ls.scal;
    gfo = sc[SC_GTP];
    fold = e.ls.armijo ? sc[SC_FOLDF] : sc[SC_FOLD];
    alpha0 = sc[SC_ALPHA0];
    accept_prev = sc[SC_ACCEPT];
    abf = abort_flag(g.abort);
  }
  sse = wave_sum_f64(sse);
  if (t < 256 && (t & 63) == 0) red[t >> 6] = sse;
  __syncthreads();
  if (t == 0) {
    const double sse_t = ((red[0] + red[1]) + red[2]) + red[3];
    const double fn = 0.5 * sse_t * e.inv_scale; // tail_fin_body's loss (lambda = 0)
    const bool fail = !ls_sufficient_decrease(e.ls, fn, fold, gfo);
    if (fail && !abf && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0) {
      double *sc = e.ls.scal;
      sc[SC_SSE] = sse_t;
      sc[SC_LOSS] = fn;
      *e.ls.abort = 1;
      SpecRecord *r = e.ls.rec;
      __hip_atomic_store(&r->loss, fn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&r->tgg, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&r->alpha0, alpha0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&r->accept_prev, accept_prev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&r->status, int(SPEC_REJECT_EARLY), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&r->seq, e.ls.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    red[4] = (abf || fail) ? 1.0 : 0.0;
  }
  __syncthreads();
  const bool out = red[4] != 0.0;
  __syncthreads(); // every wave has its verdict before any wave's first use of lds
  return out;
}

// XCD-aware placement of a split-K GEMM's blocks (cdna_hip_programming.md §5.5 T1, bijective form): blocks
// b and b + 8 are dealt to the same XCD (its own L2), so the GEMM blocks whose index e (past the side
// planes) is congruent mod 8 get one contiguous range of logical tiles, ordered split-major. The tiles of
// one split then share an L2: its A panel (the rows' input columns) is read once instead of once per
// column tile, its B panel (the rows' delta) once instead of once per row tile and XCD (784-128-10 at 7500
// rows: 77 MB of L2 misses per dW launch for 27 MB of operands, profiles/r05/i/pmc_7500.txt; 32 MB with this
// placement, dW 24.8 -> 23.4 us, profiles/r05/k/). Speed only: every logical tile is computed by exactly one
// block whatever the placement, so results do not change.
__device__ __forceinline__ void xcd_tile(int e, int n, int gx, int gy, int &z, int &bx, int &by) {
  const int q = n >> 3, r = n & 7, x = e & 7;
  const int l = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (e >> 3);
  bx = l % gx;
  by = (l / gx) % gy;
  z = l / (gx * gy);
}

// Side job (see GemmDesc): one 256-column group (four per lane) x 4 split stripes per block, fp64 in
// split order. Side blocks hold their slots for the whole launch, so a block takes many columns: 32
// loads per lane in flight per round.
constexpr int SIDE_CPL = 4;                 // columns per lane
constexpr int SIDE_COLS = 64 * SIDE_CPL;    // columns per side block
__device__ __forceinline__ void gemm_side_job(const GemmK &g, double *red) {
  const int t = threadIdx.x, lane = t & 63, stripe = t >> 6; // stripes 0-3 (extra waves idle)
  const int nside = gridDim.x * gridDim.y * g.side_planes;
  const int id = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  for (long long c0 = (long long)id * SIDE_COLS; c0 < g.side_count; c0 += (long long)nside * SIDE_COLS) {
    double acc[SIDE_CPL];
    const float *src[SIDE_CPL];
#pragma unroll
    for (int j = 0; j < SIDE_CPL; ++j) {
      const long long c = c0 + lane + 64 * j;
      acc[j] = 0.0;
      src[j] = g.side_slab + (c < g.side_count ? c : 0); // clamped; masked when stored
    }
    if (stripe < 4) {
      int k = stripe;
      for (; k + 28 < g.side_splits; k += 32) { // eight rows x four columns in flight
        float v[8][SIDE_CPL];
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
          for (int j = 0; j < SIDE_CPL; ++j) v[u][j] = src[j][(long long)(k + 4 * u) * g.side_stride];
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
          for (int j = 0; j < SIDE_CPL; ++j) acc[j] += double(v[u][j]);
      }
      for (; k < g.side_splits; k += 4)
#pragma unroll
        for (int j = 0; j < SIDE_CPL; ++j) acc[j] += double(src[j][(long long)k * g.side_stride]);
#pragma unroll
      for (int j = 0; j < SIDE_CPL; ++j) red[j * 256 + t] = acc[j];
    }
    lds_barrier();
    if (stripe == 0)
#pragma unroll
      for (int j = 0; j < SIDE_CPL; ++j) {
        const long long c = c0 + lane + 64 * j;
        const double* r = red + j * 256;
        if (c < g.side_count) g.side_dst[c] = float(((r[lane] + r[64 + lane]) + r[128 + lane]) + r[192 + lane]);
      }
    lds_barrier();
  }
}

// k-contiguous operand: R rows x 32 k. Thread chunk c -> row c>>3, k-quad c&7.
template <int R, bool GATHER>
__device__ __forceinline__ void load_kc(f32x4 (&r)[R / 32], const float *base, long long ld, const int *idx,
                                        int row0, int rows, int k0, int kend, int vec, int tid) {
#pragma unroll
  for (int i = 0; i < R / 32; ++i) {
    const int c = tid + i * 256;
    const int row = row0 + (c >> 3);
    const int k = k0 + (c & 7) * 4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (row < rows) {
      const long long grow = GATHER ? (long long)idx[row] : (long long)row;
      const float *p = base + grow * ld + k;
      if (vec && k + 3 < kend) {
        v = *reinterpret_cast<const f32x4 *>(p);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (k + j < kend) ? p[j] : 0.0f;
      }
    }
    r[i] = v;
  }
}
template <int R>
__device__ __forceinline__ void store_kc(float *lds, const f32x4 (&r)[R / 32], int tid) {
  constexpr int LDK = 36;
#pragma unroll
  for (int i = 0; i < R / 32; ++i) {
    const int c = tid + i * 256;
    *reinterpret_cast<f32x4 *>(lds + (c >> 3) * LDK + (c & 7) * 4) = r[i];
  }
}

// FAST variants (K % 4 == 0, 16-B aligned rows, cvalid % 4 == 0): every load is issued
// unconditionally from a clamped address and its value is always consumed; validity is applied when
// the tile is written to LDS (integer AND, plus the appended ones column). No divergent branches and
// no use right after the load, so the compiler counts outstanding loads (s_waitcnt vmcnt(N)) and the
// prefetched k-tiles stay in flight.
__device__ __forceinline__ f32x4 mask4(const f32x4 v, bool ok) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const unsigned m = ok ? 0xffffffffu : 0u;
  const u32x4 b = __builtin_bit_cast(u32x4, v) & (u32x4){m, m, m, m};
  return __builtin_bit_cast(f32x4, b);
}
template <int R, bool GATHER>
__device__ __forceinline__ void load_kc_fast(f32x4 (&r)[R / 32], const float *base, long long ld, const int *idx,
                                             int row0, int rows, int k0, int kend, int tid) {
#pragma unroll
  for (int i = 0; i < R / 32; ++i) {
    const int c = tid + i * 256;
    const int row = row0 + (c >> 3);
    const int k = k0 + (c & 7) * 4;
    const bool ok = row < rows && k < kend;
    const int rr = ok ? row : 0; // row 0, column 0: always a valid address
    const long long grow = GATHER ? (long long)idx[rr] : (long long)rr;
    r[i] = *reinterpret_cast<const f32x4 *>(base + grow * ld + (ok ? k : 0));
  }
}
template <int R>
__device__ __forceinline__ void store_kc_fast(float *lds, const f32x4 (&r)[R / 32], int row0, int rows, int k0,
                                              int kend, int tid) {
  constexpr int LDK = 36;
#pragma unroll
  for (int i = 0; i < R / 32; ++i) {
    const int c = tid + i * 256;
    const bool ok = row0 + (c >> 3) < rows && k0 + (c & 7) * 4 < kend;
    *reinterpret_cast<f32x4 *>(lds + (c >> 3) * LDK + (c & 7) * 4) = mask4(r[i], ok);
  }
}
template <int R, bool GATHER>
__device__ __forceinline__ void load_mc_fast(f32x4 (&r)[R / 32], const float *base, long long ld, const int *idx,
                                             int col0, int cvalid, int k0, int kend, int tid) {
  constexpr int Q = R / 4;
#pragma unroll
  for (int i = 0; i < R / 32; ++i) {
    const int c = tid + i * 256;
    const int k = k0 + c / Q;
    const int col = col0 + (c % Q) * 4;
    const bool ok = k < kend && col < cvalid;
    const int kk = ok ? k : 0; // row 0, column 0: always a valid address
    const long long grow = GATHER ? (long long)idx[kk] : (long long)kk;
    r[i] = *reinterpret_cast<const f32x4 *>(base + grow * ld + (ok ? col : 0));
  }
}
template <int R>
__device__ __forceinline__ void store_mc_fast(float *lds, const f32x4 (&r)[R / 32], int col0, int cvalid, int ones,
                                              int k0, int kend, int tid) {
  constexpr int Q = R / 4, LD = R + 4;
#pragma unroll
  for (int i = 0; i < R / 32; ++i) {
    const int c = tid + i * 256;
    const int k = k0 + c / Q;
    const int col = col0 + (c % Q) * 4;
    f32x4 v = mask4(r[i], k < kend && col < cvalid);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (k < kend && col + j == ones) v[j] = 1.0f; // appended ones column (bias row of [dW ; db])
    *reinterpret_cast<f32x4 *>(lds + (c / Q) * LD + (c % Q) * 4) = v;
  }
}

// mn-contiguous operand: 32 k-rows x R columns. Thread chunk c -> k-row c/(R/4), column quad c%(R/4).
template <int R, bool GATHER>
__device__ __forceinline__ void load_mc(f32x4 (&r)[R / 32], const float *base, long long ld, const int *idx,
                                        int col0, int cvalid, int ones, int k0, int kend, int vec, int tid) {
  constexpr int Q = R / 4;
#pragma unroll
  for (int i = 0; i < R / 32; ++i) {
    const int c = tid + i * 256;
    const int k = k0 + c / Q;
    const int col = col0 + (c % Q) * 4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (k < kend) {
      const long long grow = GATHER ? (long long)idx[k] : (long long)k;
      const float *p = base + grow * ld + col;
      if (vec && col + 3 < cvalid) {
        v = *reinterpret_cast<const f32x4 *>(p);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (col + j < cvalid) ? p[j] : ((col + j == ones) ? 1.0f : 0.0f);
      }
    }
    r[i] = v;
  }
}
template <int R>
__device__ __forceinline__ void store_mc(float *lds, const f32x4 (&r)[R / 32], int tid) {
  constexpr int Q = R / 4, LD = R + 4;
#pragma unroll
  for (int i = 0; i < R / 32; ++i) {
    const int c = tid + i * 256;
    *reinterpret_cast<f32x4 *>(lds + (c / Q) * LD + (c % Q) * 4) = r[i];
  }
}

// Epilogues shared by both main loops: the fused output layer (EPI_HEAD) or the bias/activation/
// derivative/slab store of the accumulators.
template <int WM, int WN, int TM, int TN, int EPI, int KW, class HPre>
__device__ __forceinline__ void gemm_epilogue(const GemmK &g, f32x16 (&acc)[TM][TN], float *lds, HPre &hpre, int zsplit,
                                              int m0, int n0, int wm, int wn, int li, int lh, int kgrp) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  if constexpr (EPI == EPI_HEAD) {
    KTB(1);
    // Output layer on the tile (head_core.hpp): the prefetched W / biases / targets go to LDS, then per
    // 64-row half the activations go accumulators -> LDS (bias + activation; columns >= N zero) and
    // the head runs on them. n0 == 0 (N <= BN).
    constexpr int QM = headc::qstrips(BN);
    headc::Smem hs = headc::carve(lds, g.N);
    // the head tile runs on TBR-row parts: 64-row halves, or the whole of a 32-row GEMM tile (the head's
    // products over samples then run half their steps)
    constexpr int TBR = BM < headc::TB ? BM : headc::TB;
    constexpr int YRA = BM > headc::TB ? BM : headc::TB;
    hs.xr = hs.ys + YRA * 16;
    const bool fold = g.head_fold >= 0; // uniform
    hpre.store(hs);
    if (g.head_fold > 0) hpre.store_fold(hs);
    KT(26);
    KTB(2);
    headc::f32x4 cw[QM];
#pragma unroll
    for (int q = 0; q < QM; ++q) cw[q] = (headc::f32x4){0.f, 0.f, 0.f, 0.f};
    double sse = 0.0;
    headc::TileArgs ta;
    ta.Y = g.head_Y;
    ta.idx = g.head_idx;
    ta.Out = g.head_out;
    ta.act_out = g.head_act;
    ta.act_prev = g.act;
    ta.sc = float(g.head_inv_scale);
    ta.delta = g.head_delta;
    ta.vec = (g.N & 3) == 0 && (reinterpret_cast<uintptr_t>(g.head_delta) & 15) == 0;
    ta.nfold = g.head_fold;
    headc::FoldAcc fa;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      fa.c[j] = (headc::f32x4){0.f, 0.f, 0.f, 0.f};
      fa.db[j] = 0.0f;
    }
    for (int half = 0; half < (BM + TBR - 1) / TBR; ++half) {
      const long long b0 = (long long)m0 + half * TBR;
      const int rows_tile = min(TBR, BM - half * TBR);
      const int rows = int(min((long long)rows_tile, (long long)g.M - b0));
      if (rows <= 0) break;
      ta.ys = hs.ys + half * TBR * 16;
      ta.xr = hs.xr + half * TBR * headc::XLD;
      if (half == 0) lds_barrier(); // hb (read below) written by hpre.store
      for (int e = threadIdx.x; e < (TBR - rows_tile) * hs.Hp; e += 256 * KW) { // rows the tile lacks
        const int r = rows_tile + e / hs.Hp, c = e % hs.Hp;
        hs.As[r * hs.LDA + c] = 0.0f;
      }
      with_act(g.act, [&](auto AC) __attribute__((always_inline)) {
        constexpr int A = decltype(AC)::value;
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn) {
            const int col = wn * TN * 32 + tn * 32 + li;
            const int local0 = wm * TM * 32 + tm * 32;
            if (kgrp == 0 && local0 / TBR == half && col < hs.Hp) { // the tile may be wider than Hp
              const float bn = hs.hb[col];
              const bool in = col < g.N;
#pragma unroll
              for (int r = 0; r < 16; ++r) {
                const int local = local0 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                hs.As[(local % TBR) * hs.LDA + col] = in ? act_c<A>(acc[tm][tn][r] + bn) : 0.0f;
              }
            }
          }
      });
      if (hs.Hp > BN)
        for (int e = threadIdx.x; e < rows_tile * (hs.Hp - BN); e += 256 * KW) { // padding beyond the tile width
          const int r = e / (hs.Hp - BN), c = BN + e % (hs.Hp - BN);
          hs.As[r * hs.LDA + c] = 0.0f;
        }
      lds_barrier();
      KT(28 + 2 * half);
      KTB(3 + 2 * half);
      if (fold) headc::tile<(KW > 1), QM, true, TBR>(hs, ta, b0, rows, cw, sse, fa);
      else headc::tile<(KW > 1), QM, false, TBR>(hs, ta, b0, rows, cw, sse, fa);
      KT(29 + 2 * half);
      KTB(4 + 2 * half);
    }
    KT(32);
    const long long nf = fold ? (long long)(g.head_fold + 1) * g.N : 0; // fold rows in front of the head's
    float *slab = g.head_slab + (long long)blockIdx.y * (nf + (long long)(g.N + 1) * g.head_out);
    if (fold) headc::write_fold(fa, g.N, g.head_fold, slab);
    headc::write_partials(hs, g.head_out, cw, sse, slab + nf, g.head_sse + blockIdx.y);
    KT(33);
    KTB(7);
    return;
  }
  if (KW > 1 && kgrp != 0) return; // group 0 holds the sums
  // Epilogue: lanes 0-31 own consecutive columns -> each register row is a 128-B coalesced store.
  float *C = g.C + (EPI == EPI_STORE ? (long long)zsplit * g.slab_stride : 0LL);
  // EPI_DX's act' operand (the previous layer's activations) is loaded for the whole (tm, tn) block before
  // the first use, from clamped addresses: a load-use-store per element made every element a dependent
  // memory round trip (64 per lane at 128 x 128; the cfg-3 dX GEMM spent most of its 35 us there).
  with_act(EPI == EPI_FWD ? g.act : (EPI == EPI_DX ? g.aux_act : int(ACT_LINEAR)),
           [&](auto AC) __attribute__((always_inline)) {
    constexpr int A = decltype(AC)::value;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int n = n0 + wn * TN * 32 + tn * 32 + li;
      const bool nok = n < g.N;
      float bn = 0.0f;
      if constexpr (EPI == EPI_FWD) bn = g.bias ? g.bias[nok ? n : 0] : 0.0f;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        float ax[16];
        if constexpr (EPI == EPI_DX) {
          const int nc = nok ? n : 0;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = m0 + wm * TM * 32 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
            ax[r] = g.aux[(long long)(m < g.M ? m : 0) * g.ldaux + nc];
          }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * TM * 32 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          float v = acc[tm][tn][r];
          if constexpr (EPI == EPI_FWD) v = act_c<A>(v + bn);
          if constexpr (EPI == EPI_DX) v *= dact_c<A>(ax[r]);
          if (nok && m < g.M) C[(long long)m * g.ldc + n] = v;
        }
      }
    }
  });
}

// KW k-groups of 4 waves each (KW = 2: 8 waves, two per SIMD, for tiles too small to fill the chip
// with one wave per SIMD): group q runs k-steps [16q/KW, 16(q+1)/KW) of every 32-deep tile on the
// same output sub-tile, and the groups' accumulators are summed through LDS in group order.
// PF: k-tiles whose global loads are in flight (register sets rotated in a PF-unrolled loop), so a
// load has PF compute phases to land instead of one.
template <int WM, int WN, int TM, int TN, bool AKC, bool BKC, int EPI, bool GATHER, int KW, int PF, bool FAST>
__global__ __launch_bounds__(256 * KW, 2) void gemm_kernel(const GemmK g) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32, BK = 32, LDK = BK + 4;
  constexpr int ASZ = AKC ? BM * LDK : BK * (BM + 4);
  constexpr int BSZ = BKC ? BN * LDK : BK * (BN + 4);
  constexpr int HEAD_F = headc::smem_floats_epi(BN, BM > headc::TB ? BM : headc::TB);
  constexpr int LDS_F = (EPI == EPI_HEAD && HEAD_F > 2 * (ASZ + BSZ)) ? HEAD_F : 2 * (ASZ + BSZ);
  __shared__ __attribute__((aligned(16))) float lds[LDS_F];
  if (g.early.sse_part ? gemm_early_exit(g, lds) : (g.abort && *g.abort)) return;
  if (int(blockIdx.z) < g.side_planes) {
    gemm_side_job(g, reinterpret_cast<double *>(lds));
    return;
  }
  const int zsplit = int(blockIdx.z) - g.side_planes;

  const int lane = threadIdx.x & 63, wave = (threadIdx.x >> 6) & 3, kgrp = KW > 1 ? int(threadIdx.x >> 8) : 0;
  const int wm = wave / WN, wn = wave % WN;
  const int li = lane & 31, lh = lane >> 5;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int kb = zsplit * g.k_chunk;
  const int ke = min(g.K, kb + g.k_chunk);

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;

  // staging: 256 threads per operand; with two k-groups, group 0 stages A and group 1 stages B
  const int tid = threadIdx.x & 255;
  const bool stage_a = KW == 1 || kgrp == 0, stage_b = KW == 1 || kgrp == 1;
  f32x4 ra[PF][BM / 32], rb[PF][BN / 32];
  auto gload = [&](auto &sa, auto &sb, int k0) {
    if constexpr (FAST) {
      if (stage_a) {
        if constexpr (AKC) load_kc_fast<BM, GATHER>(sa, g.A, g.lda, g.a_idx, m0, g.M, k0, ke, tid);
        else load_mc_fast<BM, GATHER>(sa, g.A, g.lda, g.a_idx, m0, g.a_mvalid, k0, ke, tid);
      }
      if (stage_b) {
        if constexpr (BKC) load_kc_fast<BN, false>(sb, g.B, g.ldb, nullptr, n0, g.N, k0, ke, tid);
        else load_mc_fast<BN, false>(sb, g.B, g.ldb, nullptr, n0, g.N, k0, ke, tid);
      }
    } else {
      if (stage_a) {
        if constexpr (AKC) load_kc<BM, GATHER>(sa, g.A, g.lda, g.a_idx, m0, g.M, k0, ke, g.a_vec, tid);
        else load_mc<BM, GATHER>(sa, g.A, g.lda, g.a_idx, m0, g.a_mvalid, g.a_ones, k0, ke, g.a_vec, tid);
      }
      if (stage_b) {
        if constexpr (BKC) load_kc<BN, false>(sb, g.B, g.ldb, nullptr, n0, g.N, k0, ke, g.b_vec, tid);
        else load_mc<BN, false>(sb, g.B, g.ldb, nullptr, n0, g.N, -1, k0, ke, g.b_vec, tid);
      }
    }
  };
  auto sstore = [&](const auto &sa, const auto &sb, int buf, int k0) {
    float *As = lds + buf * (ASZ + BSZ);
    float *Bs = As + ASZ;
    if constexpr (FAST) {
      if (stage_a) {
        if constexpr (AKC) store_kc_fast<BM>(As, sa, m0, g.M, k0, ke, tid);
        else store_mc_fast<BM>(As, sa, m0, g.a_mvalid, g.a_ones, k0, ke, tid);
      }
      if (stage_b) {
        if constexpr (BKC) store_kc_fast<BN>(Bs, sb, n0, g.N, k0, ke, tid);
        else store_mc_fast<BN>(Bs, sb, n0, g.N, -1, k0, ke, tid);
      }
      return;
    }
    if (stage_a) {
      if constexpr (AKC) store_kc<BM>(As, sa, tid);
      else store_mc<BM>(As, sa, tid);
    }
    if (stage_b) {
      if constexpr (BKC) store_kc<BN>(Bs, sb, tid);
      else store_mc<BN>(Bs, sb, tid);
    }
  };
  auto compute = [&](int buf) {
    const float *As = lds + buf * (ASZ + BSZ);
    const float *Bs = As + ASZ;
    float af[TM][AKC ? 16 : 1], bf[TN][BKC ? 16 : 1];
    if constexpr (AKC) {
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const float *p = As + (wm * TM * 32 + tm * 32 + li) * LDK + lh * 16;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 v = *reinterpret_cast<const f32x4 *>(p + q * 4);
          af[tm][q * 4 + 0] = v[0];
          af[tm][q * 4 + 1] = v[1];
          af[tm][q * 4 + 2] = v[2];
          af[tm][q * 4 + 3] = v[3];
        }
      }
    }
    if constexpr (BKC) {
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const float *p = Bs + (wn * TN * 32 + tn * 32 + li) * LDK + lh * 16;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 v = *reinterpret_cast<const f32x4 *>(p + q * 4);
          bf[tn][q * 4 + 0] = v[0];
          bf[tn][q * 4 + 1] = v[1];
          bf[tn][q * 4 + 2] = v[2];
          bf[tn][q * 4 + 3] = v[3];
        }
      }
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (KW > 1 && s / (16 / KW) != kgrp) continue; // this k-group's steps only
      float av[TM], bv[TN];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        if constexpr (AKC) av[tm] = af[tm][s];
        else av[tm] = As[(lh * 16 + s) * (BM + 4) + wm * TM * 32 + tm * 32 + li];
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        if constexpr (BKC) bv[tn] = bf[tn][s];
        else bv[tn] = Bs[(lh * 16 + s) * (BN + 4) + wn * TN * 32 + tn * 32 + li];
      }
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[tm], bv[tn], acc[tm][tn], 0, 0, 0);
    }
  };

  if (EPI == EPI_HEAD) KT(0);
  if (EPI == EPI_HEAD) KTB(0);
  if (EPI == EPI_HEAD) KTHW();
  // EPI_HEAD: the head's HBM inputs (W, biases, targets) are loaded while the last k-tile computes
  headc::EpiPrefetch<BN, BM, 256 * KW> hpre;
  if (kb < ke) {
    const int nk = (ke - kb + BK - 1) / BK;
    const int nloop = EPI == EPI_HEAD ? nk - 1 : nk; // EPI_HEAD peels the last k-tile
    // register set p holds k-tile i with i % PF == p; LDS buffer i & 1 holds k-tile i while computed
#pragma unroll
    for (int p = 0; p < PF; ++p)
      if (p < nk) gload(ra[p], rb[p], kb + p * BK);
    sstore(ra[0], rb[0], 0, kb);
    __syncthreads();
    for (int i0 = 0; i0 < nloop; i0 += PF) {
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const int i = i0 + u;
        if (i >= nloop) break;
        if (PF > 1 && i + PF < nk) gload(ra[u], rb[u], kb + (i + PF) * BK); // set u's tile i is in LDS
        if (PF == 1 && i + 1 < nk) gload(ra[0], rb[0], kb + (i + 1) * BK);
        compute(i & 1);
        if (i + 1 < nk) sstore(ra[(u + 1) % PF], rb[(u + 1) % PF], (i + 1) & 1, kb + (i + 1) * BK);
        __syncthreads();
        if (EPI == EPI_HEAD && i < 24) KT(1 + i);
      }
    }
    if constexpr (EPI == EPI_HEAD) {
      hpre.load(g.head_P, g.N, g.head_out, g.bias, g.head_Y, g.head_idx, m0, g.M);
      if (g.head_fold > 0) hpre.load_fold(g.A, g.lda, g.a_idx, g.head_fold_c0, g.head_fold, m0, g.M);
      compute((nk - 1) & 1);
      __syncthreads();
      KT(25);
    }
  } else if constexpr (EPI == EPI_HEAD) {
    hpre.load(g.head_P, g.N, g.head_out, g.bias, g.head_Y, g.head_idx, m0, g.M);
    if (g.head_fold > 0) hpre.load_fold(g.A, g.lda, g.a_idx, g.head_fold_c0, g.head_fold, m0, g.M);
  }
  if constexpr (KW > 1) { // group sums through LDS, in group order (group 0 keeps the result)
    float *red = lds;
    constexpr int PER = TM * TN * 16;
    for (int q = 1; q < KW; ++q) {
      if (kgrp == q) {
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) red[((a * TN + b) * 16 + r) * 256 + (threadIdx.x & 255)] = acc[a][b][r];
      }
      __syncthreads();
      if (kgrp == 0) {
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] += red[((a * TN + b) * 16 + r) * 256 + threadIdx.x];
      }
      __syncthreads();
    }
    static_assert(PER * 256 <= LDS_F, "k-group reduction buffer");
  }

  gemm_epilogue<WM, WN, TM, TN, EPI, KW>(g, acc, lds, hpre, zsplit, m0, n0, wm, wn, li, lh, kgrp);
}

// ------------------------------------------------------------------------------------------------
// LDS-DMA main loop (global_load_lds_dwordx4): operand tiles go HBM -> LDS with no register staging,
// NS tile buffers in a ring, NS-1 k-tiles in flight. Each wave issues the same P = (BM+BN)/32 1-KiB
// pieces per k-tile, so "k-tile i has landed" is a counted s_waitcnt vmcnt(P * tiles issued after
// it) plus a raw s_barrier (a __syncthreads would drain every tile in flight).
// The DMA writes 64 lanes x 16 B contiguously, so the LDS images are unpadded and the bank-conflict
// swizzle is applied through the per-lane SOURCE address:
//   k-contiguous [R][32]: 16-B chunk slot c of row r holds global chunk c ^ ((r >> 1) & 7)
//       (a ds_read_b128 quarter-wave covers 16 distinct bank groups);
//   mn-contiguous [32][R] (R >= 64): row k holds its chunks XOR 8 when k >= 16 (column ^ 32), so the
//       two lane halves (k = s and k = 16 + s) of a ds_read_b32 use opposite bank halves.
// Out-of-range chunks (rows >= M, k >= K, columns >= N) read a zero chunk; the bias "ones" column reads
// {1,0,0,0}. Requires K % 4 == 0, 16-B aligned rows and column counts % 4 == 0 (FAST shapes).
// ------------------------------------------------------------------------------------------------
__device__ __attribute__((aligned(16))) const float lbf_glds_const[8] = {0.f, 0.f, 0.f, 0.f, 1.f, 0.f, 0.f, 0.f};

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

__device__ __forceinline__ void glds16(const float *src, float *lds_dst) {
  __builtin_amdgcn_global_load_lds((glb_void_t *)src, (lds_void_t *)lds_dst, 16, 0, 0);
}
template <int N> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// wait until at most `ahead` k-tiles (P pieces each) of this wave are still in flight
template <int P, int NS> __device__ __forceinline__ void vm_wait_tiles(int ahead) {
  static_assert(NS >= 2 && NS <= 6, "stages");
  if (NS >= 6 && ahead >= 4) vm_wait<4 * P>();
  else if (NS >= 5 && ahead >= 3) vm_wait<3 * P>();
  else if (NS >= 4 && ahead >= 2) vm_wait<2 * P>();
  else if (NS >= 3 && ahead >= 1) vm_wait<P>();
  else vm_wait<0>();
}

// One 1-KiB piece of a k-tile: per-lane source for k-tile t.
struct GldsPiece {
  unsigned long long p0; // source address at the block's first k-tile (the zero / ones chunk if out of range)
  unsigned long long step; // bytes per k-tile (0 for the constant chunks)
  int kq;                  // k offset of this lane's chunk / row inside a k-tile
};

// KW = 2 (small tiles that run one workgroup per CU, e.g. 32 x 128 for a rank's shard): eight waves, two
// per SIMD; k-group q computes steps [8q, 8q+8) of every 32-deep tile from the same LDS stage, group 0
// alone issues the LDS-DMA pieces, and the groups' accumulators are summed through LDS in group order.
template <int WM, int WN, int TM, int TN, int EPI, int NS> struct GldsShape {
  static constexpr int BM = WM * TM * 32, BN = WN * TN * 32, BK = 32;
  static constexpr int STG = (BM + BN) * BK;
  static constexpr int HEAD_F = headc::smem_floats_epi(BN, BM > headc::TB ? BM : headc::TB);
  static constexpr int LDS_F = (EPI == EPI_HEAD && HEAD_F > NS * STG) ? HEAD_F : NS * STG;
};

// One GEMM tile (bx, by) of split zsplit (the kernels below choose the problem and the tile).
template <int WM, int WN, int TM, int TN, bool AKC, bool BKC, int EPI, bool GATHER, int NS, int KW, bool ASUM>
__device__ __forceinline__ void glds_body(const GemmK &g, float *lds, int zsplit, int bx, int by) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32, BK = 32;
  constexpr int ASZ = BM * BK, STG = (BM + BN) * BK;
  constexpr int PA = BM / 8, P = (BM + BN) / 32; // A pieces per k-tile, pieces per wave per k-tile
  static_assert((BM + BN) % 32 == 0, "pieces per wave");
  static_assert(AKC || BM >= 64, "mn-contiguous swizzle needs >= 64 columns");
  static_assert(BKC || BN >= 64, "mn-contiguous swizzle needs >= 64 columns");
  static_assert(!ASUM || (AKC && !GATHER && PA == 4), "A from slabs: the 32-row k-contiguous tile, one A piece per wave");
  constexpr int PD = ASUM ? P - 1 : P; // LDS-DMA pieces per wave per k-tile
  constexpr int LDS_F = GldsShape<WM, WN, TM, TN, EPI, NS>::LDS_F;
  const int lane = threadIdx.x & 63, wave = (threadIdx.x >> 6) & 3;
  const int kgrp = KW > 1 ? __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 8)) : 0;
  const int wm = wave / WN, wn = wave % WN;
  const int li = lane & 31, lh = lane >> 5;
  const int n0 = bx * BN, m0 = by * BM;
  const int kb = zsplit * g.k_chunk;
  const int ke = min(g.K, kb + g.k_chunk);

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;

  // ---- this wave's pieces: j = wave + 4 i; j < PA -> A, else B (k-group 0 only) ----
  const unsigned long long zero_u = reinterpret_cast<unsigned long long>(lbf_glds_const);
  GldsPiece pc[P];
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const int j = wave + 4 * i;
    const bool isA = j < PA;
    const int jj = isA ? j : j - PA;
    const bool kc = isA ? AKC : BKC;
    const float *base = isA ? g.A : g.B;
    const long long ld = isA ? g.lda : g.ldb;
    GldsPiece q;
    bool ok, ones = false;
    const float *src;
    if (kc) { // rows 8jj .. 8jj+7, 8 chunks each
      const int r = 8 * jj + (lane >> 3);
      const int gc = (lane & 7) ^ ((r >> 1) & 7);
      const int row = (isA ? m0 : n0) + r;
      ok = row < (isA ? g.M : g.N);
      long long grow = ok ? row : 0;
      if (GATHER && isA && ok) grow = g.a_idx[row];
      src = base + grow * ld + kb + 4 * gc;
      q.step = BK * sizeof(float);
      q.kq = 4 * gc;
    } else { // R columns per k-row, 256 / R k-rows per piece
      const int R = isA ? BM : BN;
      const int kl = jj * (256 / R) + (lane * 4) / R;
      const int gc = ((lane * 4) % R / 4) ^ (((kl >> 4) & 1) * 8);
      const int col = (isA ? m0 : n0) + 4 * gc;
      ok = col < (isA ? g.a_mvalid : g.N);
      ones = isA && col == g.a_ones;
      src = base + (long long)(kb + kl) * ld + (ok ? col : 0);
      q.step = (unsigned long long)(BK * ld) * sizeof(float);
      q.kq = kl;
    }
    q.p0 = ok ? reinterpret_cast<unsigned long long>(src) : zero_u + (ones ? 16 : 0);
    if (!ok) q.step = 0;
    pc[i] = q;
  }
  auto issue = [&](int t) {
    if (KW > 1 && kgrp != 0) return; // wave-uniform
    float *stage = lds + (t % NS) * STG;
    const int kt = kb + t * BK;
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const int j = wave + 4 * i;
      if (ASUM && j < PA) continue; // formed by the prologue
      const unsigned long long a = pc[i].p0 + (unsigned long long)t * pc[i].step;
      glds16(reinterpret_cast<const float *>(kt + pc[i].kq < ke ? a : zero_u),
             stage + (j < PA ? j * 256 : ASZ + (j - PA) * 256));
    }
  };
  // fragments of one k-tile for this k-group: 16 / KW k-steps of every (tm, tn) operand
  constexpr int KWC = KW; // k-groups sharing the MFMA work
  const int kq0 = kgrp;
  constexpr int SK = 16 / KWC;
  struct Frag {
    float a[TM][SK], b[TN][SK];
  };
  auto lds_frag = [&](int buf, Frag &f) {
    const float *As = lds + buf * STG;
    const float *Bs = As + ASZ;
    constexpr int QW = 4 / KWC; // 16-B quads of the k-contiguous fragments this k-group consumes
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      const int row = wm * TM * 32 + tm * 32 + li;
      if constexpr (AKC) {
        const int sw = (row >> 1) & 7;
#pragma unroll
        for (int qq = 0; qq < QW; ++qq) {
          const int q = kq0 * QW + qq;
          const f32x4 v = *reinterpret_cast<const f32x4 *>(As + row * BK + 4 * ((lh * 4 + q) ^ sw));
#pragma unroll
          for (int e = 0; e < 4; ++e) f.a[tm][qq * 4 + e] = v[e];
        }
      } else {
#pragma unroll
        for (int ss = 0; ss < SK; ++ss) f.a[tm][ss] = As[(lh * 16 + kq0 * SK + ss) * BM + (row ^ (lh << 5))];
      }
    }
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int row = wn * TN * 32 + tn * 32 + li;
      if constexpr (BKC) {
        const int sw = (row >> 1) & 7;
#pragma unroll
        for (int qq = 0; qq < QW; ++qq) {
          const int q = kq0 * QW + qq;
          const f32x4 v = *reinterpret_cast<const f32x4 *>(Bs + row * BK + 4 * ((lh * 4 + q) ^ sw));
#pragma unroll
          for (int e = 0; e < 4; ++e) f.b[tn][qq * 4 + e] = v[e];
        }
      } else {
#pragma unroll
        for (int ss = 0; ss < SK; ++ss) f.b[tn][ss] = Bs[(lh * 16 + kq0 * SK + ss) * BN + (row ^ (lh << 5))];
      }
    }
  };
  auto mfma_frag = [&](const Frag &f) {
#pragma unroll
    for (int ss = 0; ss < SK; ++ss)
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(f.a[tm][ss], f.b[tn][ss], acc[tm][tn], 0, 0, 0);
  };
  auto compute = [&](int buf) {
    Frag f;
    lds_frag(buf, f);
    mfma_frag(f);
  };

  if (EPI == EPI_HEAD) KT(0);
  if (EPI == EPI_HEAD) KTC(40);
  if (EPI == EPI_HEAD) KTB(0);
  if (EPI == EPI_HEAD) KTHW();
  headc::EpiPrefetch<BN, BM, 256 * KW> hpre;
  if constexpr (EPI == EPI_HEAD) {
    hpre.load(g.head_P, g.N, g.head_out, g.bias, g.head_Y, g.head_idx, m0, g.M);
    if (g.head_fold > 0) hpre.load_fold(g.A, g.lda, g.a_idx, g.head_fold_c0, g.head_fold, m0, g.M);
  }
  const int nk = kb < ke ? (ke - kb + BK - 1) / BK : 0;
  if constexpr (ASUM) {
    // This wave's A piece (rows 8 wave .. +7, the DMA's chunk swizzle) of every k-tile of the chunk (nk <= NS,
    // gemm_asum_ok), k-tile t by k-group t % KW: all splits' 16-B quads loaded, summed in split order (fp32,
    // fwd_reduce_act's order), + bias, activation, into the tile's stage; rows / k past the ends are zeros,
    // as the DMA's zero chunk. Column tile 0 also stores the activations.
    const int r = 8 * wave + (lane >> 3);
    const int gc = (lane & 7) ^ ((r >> 1) & 7);
    const int row = m0 + r;
    const bool rok = row < g.M;
    const long long rbase = (long long)(rok ? row : 0) * g.lda;
    for (int t = kgrp; t < nk; t += KW) {
      const int kq = kb + t * BK + 4 * gc;
      const bool ok = rok && kq < ke;
      const long long off = rbase + (ok ? kq : 0);
      f32x4 sum = {0.f, 0.f, 0.f, 0.f};
      for (int s0 = 0; s0 < g.a_splits; s0 += 8) {
        f32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) { // unconditional (clamped split), masked in the sum
          const int sp = min(s0 + u, g.a_splits - 1);
          v[u] = *reinterpret_cast<const f32x4 *>(g.a_slab + (long long)sp * g.a_slab_stride + off);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (s0 + u < g.a_splits) sum += v[u];
      }
      const f32x4 b4 = *reinterpret_cast<const f32x4 *>(g.a_bias + (ok ? kq : 0));
      f32x4 a4;
#pragma unroll
      for (int e = 0; e < 4; ++e) a4[e] = ok ? act_rt(g.a_act, sum[e] + b4[e]) : 0.0f;
      *reinterpret_cast<f32x4 *>(lds + (t % NS) * STG + wave * 256 + lane * 4) = a4;
      if (ok && bx == 0) *reinterpret_cast<f32x4 *>(g.a_out + rbase + kq) = a4;
    }
  }
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nk) issue(t);
  {
    for (int i = 0; i < nk; ++i) {
      vm_wait_tiles<PD, NS>(min(NS - 2, nk - 1 - i)); // this wave's pieces of k-tile i landed
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier(); // everyone's pieces landed; buffer (i - 1) % NS no longer read
      if (EPI == EPI_HEAD && i < 24) KT(1 + i);
      if (i + NS - 1 < nk) issue(i + NS - 1);
      compute(i % NS);
    }
  }
  if (EPI == EPI_HEAD) KT(25);
  if (EPI == EPI_HEAD) KTC(41);
  __syncthreads(); // the LDS is the epilogue's now
  if constexpr (KW > 1) { // group sums through LDS, in group order (group 0 keeps the result)
    float *red = lds;
    static_assert(TM * TN * 16 * 256 <= LDS_F, "k-group reduction buffer");
    for (int q = 1; q < KW; ++q) {
      if (kgrp == q) {
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) red[((a * TN + b) * 16 + r) * 256 + (threadIdx.x & 255)] = acc[a][b][r];
      }
      __syncthreads();
      if (kgrp == 0) {
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] += red[((a * TN + b) * 16 + r) * 256 + threadIdx.x];
      }
      __syncthreads();
    }
  }
  gemm_epilogue<WM, WN, TM, TN, EPI, KW>(g, acc, lds, hpre, zsplit, m0, n0, wm, wn, li, lh, kgrp);
}

template <int WM, int WN, int TM, int TN, bool AKC, bool BKC, int EPI, bool GATHER, int NS, int KW = 1, bool ASUM = false>
__global__ __launch_bounds__(256 * KW, KW == 1 ? 2 : 1) void gemm_glds_kernel(const GemmK g) {
  __shared__ __attribute__((aligned(16))) float lds[GldsShape<WM, WN, TM, TN, EPI, NS>::LDS_F];
  if (g.early.sse_part ? gemm_early_exit(g, lds) : (g.abort && *g.abort)) return;
  if (int(blockIdx.z) < g.side_planes) {
    gemm_side_job(g, reinterpret_cast<double *>(lds));
    return;
  }
  int z = int(blockIdx.z) - g.side_planes, bx = int(blockIdx.x), by = int(blockIdx.y);
  if (g.xcd_swz) {
    const int plane = int(gridDim.x * gridDim.y);
    xcd_tile(z * plane + by * int(gridDim.x) + bx, (int(gridDim.z) - g.side_planes) * plane, int(gridDim.x),
             int(gridDim.y), z, bx, by);
  }
  glds_body<WM, WN, TM, TN, AKC, BKC, EPI, GATHER, NS, KW, ASUM>(g, lds, z, bx, by);
}

// Two GEMMs of one shape in one launch (the S-LBFGS minibatch's dW GEMMs of adjacent layers): planes
// [0, side_planes) run g's side job, the next g.group_z planes g's splits, the rest g2's; a block past its
// problem's tile grid exits.
template <int WM, int WN, int TM, int TN, bool AKC, bool BKC, int EPI, int NS, int KW = 1>
__global__ __launch_bounds__(256 * KW, KW == 1 ? 2 : 1) void gemm_glds_group_kernel(const GemmK g, const GemmK g2) {
  __shared__ __attribute__((aligned(16))) float lds[GldsShape<WM, WN, TM, TN, EPI, NS>::LDS_F];
  if (g.early.sse_part ? gemm_early_exit(g, lds) : (g.abort && *g.abort)) return;
  if (int(blockIdx.z) < g.side_planes) {
    gemm_side_job(g, reinterpret_cast<double *>(lds));
    return;
  }
  const int z = int(blockIdx.z) - g.side_planes, bx = int(blockIdx.x), by = int(blockIdx.y);
  if (z >= g.group_z) {
    if (bx >= g2.gx || by >= g2.gy) return;
    glds_body<WM, WN, TM, TN, AKC, BKC, EPI, false, NS, KW, false>(g2, lds, z - g.group_z, bx, by);
  } else {
    if (bx >= g.gx || by >= g.gy) return;
    glds_body<WM, WN, TM, TN, AKC, BKC, EPI, false, NS, KW, false>(g, lds, z, bx, by);
  }
}

// ------------------------------------------------------------------------------------------------
// Wave-split-K direct-load main loop for the 32 x 128 tile (round 5; microbenchmark profiles/micro/loop32.hip,
// whose results were lost with the session that ran it; library A/B in profiles/r05/g/, n/). The LDS-DMA loop of this tile spends ~1.8k cycles per 32-deep k-tile against 1024 of MFMA
// issue: its DMA writes and fragment reads contend for the LDS while each wave waits on its reads, and the
// DMA pieces' issue cost sits in front of the MFMAs. Here no operand is shared between waves and nothing
// goes through LDS until the end: the four waves split every 32-deep k-tile (wave w: k 8w .. 8w+7, lane half
// h: the 4 consecutive k 8w+4h .. +3), each lane loads its A quad A[row][k..k+3] and, per k, one 16-B quad of
// the B row (columns n0 + 4 li .. +3) straight into registers, WSK_PD k-tiles ahead. The quad's 4 columns feed
// 4 accumulators (accumulator c holds columns n0 + 4 j + c), 16 v_mfma_f32_32x32x2_f32 per wave per k-tile on 4
// independent chains. After the loop the four waves' partial tiles are summed in wave order through LDS into
// the standard accumulator layout (wave w owns columns n0 + 32w .. +31), so the epilogues (bias + activation,
// split-K slab, the fused output layer) are the LDS-DMA kernel's. Fixed order throughout: a re-evaluation is
// bitwise identical. Requires K, lda, ldb, N, k_chunk % 4 == 0 and 16-B aligned A, B (wsk_ok).
// ------------------------------------------------------------------------------------------------
constexpr int WSK_PD = 3;
constexpr int WSK_RED_F = 4 * 16 * 2 * 128; // four waves' partial tiles, [wave][r][h][128 columns]
constexpr int WSK_MAX_ASPLITS = 8;          // A-from-slabs: splits summed per quad (gemm_wsk_ok)

// BKC: B stored k-contiguous (B[n*ldb + k]: the dX GEMM's W^T): a lane loads, per column block c, the quad
// B[n0 + 32c + li][k..k+3], and accumulator c holds the standard columns n0 + 32c + j. Else (B n-contiguous)
// the lane loads, per k, the quad B[k][n0 + 4li .. +3], and accumulator c holds columns n0 + 4j + c.
// ASUM: the A quad is act(sum over the previous layer's forward split-K slabs in split order + bias) (the
// LDS-DMA kernel's prologue and fwd_reduce_act's arithmetic), and the workgroups of column tile 0 store it to
// a_out for the backward phase.
template <int EPI, bool GATHER, bool BKC, bool ASUM>
__global__ __launch_bounds__(256, 1) void gemm_wsk_kernel(const GemmK g) {
  constexpr int BM = 32, BN = 128;
  constexpr int HEAD_F = headc::smem_floats_epi(BN, headc::TB);
  constexpr int LDS_F = HEAD_F > WSK_RED_F ? HEAD_F : WSK_RED_F;
  constexpr int NA = ASUM ? WSK_MAX_ASPLITS : 1; // A quads per k-tile
  __shared__ __attribute__((aligned(16))) float lds[LDS_F];
  if (g.early.sse_part ? gemm_early_exit(g, lds) : (g.abort && *g.abort)) return;
  if (int(blockIdx.z) < g.side_planes) {
    gemm_side_job(g, reinterpret_cast<double *>(lds));
    return;
  }
  const int zsplit = int(blockIdx.z) - g.side_planes;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int m0 = int(blockIdx.y) * BM, n0 = int(blockIdx.x) * BN;
  const int kb = zsplit * g.k_chunk;
  const int ke = min(g.K, kb + g.k_chunk);
  headc::EpiPrefetch<BN, BM, 256> hpre;
  if constexpr (EPI == EPI_HEAD) {
    hpre.load(g.head_P, g.N, g.head_out, g.bias, g.head_Y, g.head_idx, m0, g.M);
    if (g.head_fold > 0) hpre.load_fold(g.A, g.lda, g.a_idx, g.head_fold_c0, g.head_fold, m0, g.M);
  }
  // rows past M and columns past N read row 0 / column n0 (finite data); the epilogues mask them
  const int row = m0 + li;
  const bool rok = row < g.M;
  long long grow = rok ? row : 0;
  if (GATHER && rok) grow = g.a_idx[row];
  const int k4 = 8 * wave + 4 * lh;
  const float *ap = (ASUM ? g.a_slab : g.A) + grow * g.lda + kb + k4;
  const float *bp[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if constexpr (BKC) {
      const int n = n0 + 32 * c + li;
      bp[c] = g.B + (long long)(n < g.N ? n : n0) * g.ldb + kb + k4;
    } else {
      const int col = n0 + 4 * li;
      bp[c] = g.B + (long long)(kb + k4 + c) * g.ldb + (col < g.N ? col : n0); // c: the k within the quad
    }
  }
  const int nk = kb < ke ? (ke - kb + 31) / 32 : 0;
  f32x16 acc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.0f;
  f32x4 ra[WSK_PD][NA], rb[WSK_PD][4], rbias[WSK_PD];
  bool okm[WSK_PD];
  // k-tile tt into register slot `slot`: clamped and unconditional (a k quad is all in or all out of
  // [kb, ke): k4, kb, ke are multiples of 4); the mask is applied at the use
  auto load = [&](int tt, int slot) {
    const bool ok = kb + tt * 32 + k4 < ke;
    const long long ko = ok ? (long long)tt * 32 : 0;
    okm[slot] = ok;
    if constexpr (ASUM) {
#pragma unroll
      for (int u = 0; u < NA; ++u) // every split's quad (clamped split; masked in the sum)
        ra[slot][u] = *reinterpret_cast<const f32x4 *>(ap + (long long)min(u, g.a_splits - 1) * g.a_slab_stride + ko);
      rbias[slot] = *reinterpret_cast<const f32x4 *>(g.a_bias + kb + k4 + ko);
    } else {
      ra[slot][0] = *reinterpret_cast<const f32x4 *>(ap + ko);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
      rb[slot][c] = *reinterpret_cast<const f32x4 *>(bp[c] + (BKC ? ko : ko * g.ldb));
  };
#pragma unroll
  for (int p = 0; p < WSK_PD; ++p) load(p, p);
  for (int i0 = 0; i0 < nk; i0 += WSK_PD) {
#pragma unroll
    for (int p = 0; p < WSK_PD; ++p) {
      const int i = i0 + p;
      if (i < nk) { // wave-uniform
        f32x4 a;
        if constexpr (ASUM) {
          f32x4 sum = ra[p][0];
#pragma unroll
          for (int u = 1; u < NA; ++u)
            if (u < g.a_splits) sum += ra[p][u];
#pragma unroll
          for (int e = 0; e < 4; ++e) a[e] = act_rt(g.a_act, sum[e] + rbias[p][e]);
          if (okm[p] && rok && n0 == 0) // column tile 0 stores the activations (bitwise fwd_reduce_act's)
            *reinterpret_cast<f32x4 *>(g.a_out + (long long)row * g.lda + kb + k4 + (long long)i * 32) = a;
        } else {
          a = ra[p][0];
        }
        if (!okm[p]) a = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int c = 0; c < 4; ++c)
            acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q], BKC ? rb[p][c][q] : rb[p][q][c], acc[c], 0, 0, 0);
      }
      // the slot's next k-tile, issued after the MFMAs that read it (no register copy, so no wait for the new
      // data in this iteration): WSK_PD - 1 k-tiles of MFMAs ahead of its use
      __builtin_amdgcn_sched_barrier(0);
      load(i + WSK_PD, p);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // the partial tiles, summed in wave order, into the standard layout (wave w: columns 32w + j)
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float *dst = &lds[((wave * 16 + r) * 2 + lh) * 128];
    if constexpr (BKC) {
#pragma unroll
      for (int c = 0; c < 4; ++c) dst[32 * c + li] = acc[c][r];
    } else {
      *reinterpret_cast<f32x4 *>(dst + li * 4) = f32x4{acc[0][r], acc[1][r], acc[2][r], acc[3][r]};
    }
  }
  __syncthreads();
  f32x16 out[1][1];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float v = lds[((0 * 16 + r) * 2 + lh) * 128 + 32 * wave + li];
#pragma unroll
    for (int w = 1; w < 4; ++w) v += lds[((w * 16 + r) * 2 + lh) * 128 + 32 * wave + li];
    out[0][0][r] = v;
  }
  __syncthreads(); // the LDS is the epilogue's now
  gemm_epilogue<1, 4, 1, 1, EPI, 1>(g, out, lds, hpre, zsplit, m0, n0, 0, wave, li, lh, 0);
}

namespace {

bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

template <int BM, int BN> GemmK make_gemmk(const GemmDesc &d) {
  GemmK k;
  k.M = d.M;
  k.N = d.N;
  k.K = d.K;
  k.k_chunk = d.splits > 1 ? d.k_chunk : d.K;
  k.A = d.A;
  k.lda = d.lda;
  k.a_idx = d.a_idx;
  k.a_mvalid = d.a_mvalid > 0 ? d.a_mvalid : d.M;
  k.a_ones = d.a_ones;
  k.a_vec = (d.lda % 4 == 0) && aligned16(d.A);
  k.B = d.B;
  k.ldb = d.ldb;
  k.b_vec = (d.ldb % 4 == 0) && aligned16(d.B);
  k.C = d.C;
  k.ldc = d.ldc;
  k.slab_stride = d.slab_stride;
  k.bias = d.bias;
  k.act = d.act;
  k.aux = d.aux;
  k.ldaux = d.ldaux;
  k.aux_act = d.aux_act;
  k.abort = d.abort;
  if (d.early) k.early = *d.early;
  const long long gx = (d.N + BN - 1) / BN, gy = (d.M + BM - 1) / BM;
  k.gx = int(gx);
  k.gy = int(gy);
  k.group_z = 0;
  static const bool xcd_off = [] { // A/B switch: LBF_NO_XCD=1 keeps the default block placement
    const char *e = std::getenv("LBF_NO_XCD");
    return e && std::atoi(e) != 0;
  }();
  // dW GEMMs only (A = activations^T, mn-contiguous). The split-K FORWARD of a minibatch (config 4's
  // 256 x 784 -> 512, 32 x 128 tiles, 8 splits) measured slower with it: 12.3 -> 13.2-13.7 us per launch for
  // 10.2 -> 7.9 MB of traffic (every CU of an XCD then streams the same W chunk at once); profiles/r05/k/.
  k.xcd_swz = !xcd_off && d.epi == EPI_STORE && d.splits > 1 && !d.a_kc;
  k.side_planes = (d.side_slab && d.side_count > 0) ? int(cdiv(cdiv(d.side_count, SIDE_COLS), gx * gy)) : 0;
  k.side_slab = d.side_slab;
  k.side_splits = d.side_splits;
  k.side_stride = d.side_stride;
  k.side_count = d.side_count;
  k.side_dst = d.side_dst;
  k.head_P = d.head_P;
  k.head_out = d.head_out;
  k.head_act = d.head_act;
  k.head_Y = d.head_Y;
  k.head_idx = d.head_idx;
  k.head_inv_scale = d.head_inv_scale;
  k.head_delta = d.head_delta;
  k.head_slab = d.head_slab;
  k.head_sse = d.head_sse;
  k.head_fold = d.head_fold;
  k.head_fold_c0 = d.head_fold_c0;
  k.a_slab = d.a_slab;
  k.a_splits = d.a_splits;
  k.a_slab_stride = d.a_slab_stride;
  k.a_bias = d.a_bias;
  k.a_act = d.a_act;
  k.a_out = d.a_out;
  return k;
}

// NS > 0: the LDS-DMA kernel with NS tile buffers where the shape allows it (FAST shapes, no gathered
// mn-contiguous operand); otherwise the register-staged kernel (KW k-groups, PF register sets).
template <int WM, int WN, int TM, int TN, bool AKC, bool BKC, int EPI, int KW = 1, int PF = 1, int NS = 0>
void launch(hipStream_t s, const GemmDesc &d, const GemmDesc *d2 = nullptr) {
  // FAST loads: K % 4 == 0, vector-aligned operands, column counts % 4 == 0
  const bool fast = d.K % 4 == 0 && (d.lda % 4 == 0) && (d.ldb % 4 == 0) &&
                    ((reinterpret_cast<uintptr_t>(d.A) | reinterpret_cast<uintptr_t>(d.B)) & 15) == 0 &&
                    (AKC || (d.a_mvalid > 0 ? d.a_mvalid : d.M) % 4 == 0) && (BKC || d.N % 4 == 0);
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  GemmK k = make_gemmk<BM, BN>(d);
  const long long gx = k.gx, gy = k.gy;
  dim3 grid(unsigned(gx), unsigned(gy), unsigned((d.splits > 1 ? d.splits : 1) + k.side_planes));
  if (d2) { // grouped with a second problem of this shape (gemm_group_ok): its splits follow d's
    if constexpr (NS > 0 && (AKC || BM >= 64) && (BKC || BN >= 64)) {
      GemmDesc e = *d2;
      e.side_slab = nullptr;
      e.side_count = 0;
      GemmK k2 = make_gemmk<BM, BN>(e);
      k.group_z = d.splits > 1 ? d.splits : 1;
      const long long gx2 = std::max<long long>(gx, k2.gx), gy2 = std::max<long long>(gy, k2.gy);
      k.side_planes = (d.side_slab && d.side_count > 0) ? int(cdiv(cdiv(d.side_count, SIDE_COLS), gx2 * gy2)) : 0;
      const dim3 g3(unsigned(gx2), unsigned(gy2), unsigned(k.group_z + (e.splits > 1 ? e.splits : 1) + k.side_planes));
      hipLaunchKernelGGL((gemm_glds_group_kernel<WM, WN, TM, TN, AKC, BKC, EPI, NS, KW>), g3, dim3(256 * KW), 0, s, k,
                         k2);
      return;
    }
    throw std::runtime_error("gemm: grouped launch not supported for this tile");
  }
  if constexpr (NS > 0 && (AKC || BM >= 64) && (BKC || BN >= 64)) { // mn-contiguous swizzle: >= 64 columns
    if (fast && (AKC || !d.a_idx)) {
      const dim3 gb(256 * KW);
      if constexpr (AKC && BM == 32 && WN * TN == 4 && NS >= 2) {
        if (d.a_slab) { // gemm_asum_ok
          hipLaunchKernelGGL((gemm_glds_kernel<WM, WN, TM, TN, AKC, BKC, EPI, false, NS, KW, true>), grid, gb, 0, s, k);
          return;
        }
      }
      if (d.a_slab) throw std::runtime_error("gemm: A from slabs not supported for this tile");
      if (d.a_idx)
        hipLaunchKernelGGL((gemm_glds_kernel<WM, WN, TM, TN, AKC, BKC, EPI, true, NS, KW>), grid, gb, 0, s, k);
      else
        hipLaunchKernelGGL((gemm_glds_kernel<WM, WN, TM, TN, AKC, BKC, EPI, false, NS, KW>), grid, gb, 0, s, k);
      return;
    }
  }
  const dim3 block(256 * KW);
  if (fast) {
    if (d.a_idx) hipLaunchKernelGGL((gemm_kernel<WM, WN, TM, TN, AKC, BKC, EPI, true, KW, PF, true>), grid, block, 0, s, k);
    else hipLaunchKernelGGL((gemm_kernel<WM, WN, TM, TN, AKC, BKC, EPI, false, KW, PF, true>), grid, block, 0, s, k);
  } else { // general shapes: guarded loads, one k-tile in flight
    if (d.a_idx) hipLaunchKernelGGL((gemm_kernel<WM, WN, TM, TN, AKC, BKC, EPI, true, KW, 1, false>), grid, block, 0, s, k);
    else hipLaunchKernelGGL((gemm_kernel<WM, WN, TM, TN, AKC, BKC, EPI, false, KW, 1, false>), grid, block, 0, s, k);
  }
}

// gemm_wsk_kernel's conditions: 16-B quads everywhere. Opt-in (LBF_WSK=1): in the library's GEMMs it measured
// no faster than the LDS-DMA loop at the 8-rank shard's fused-head forward and 10 % slower on config 4's
// minibatch GEMMs (profiles/r05/g/), although its main loop alone measured 28 % faster (profiles/micro/loop32.hip).
static bool wsk_ok(const GemmDesc &d) {
  static const bool off = [] {
    const char *e = std::getenv("LBF_WSK");
    return !(e && std::atoi(e) != 0);
  }();
  const int kc = d.splits > 1 ? d.k_chunk : d.K;
  const bool base = !off && d.a_kc && d.K % 4 == 0 && d.lda % 4 == 0 && d.ldb % 4 == 0 && kc % 4 == 0 &&
                    aligned16(d.A) && aligned16(d.B);
  if (!base) return false;
  if (d.a_slab) // A from the previous layer's slabs: forward operand layout, split-K store or plain forward
    return !d.b_kc && !d.a_idx && (d.epi == EPI_STORE || d.epi == EPI_FWD) && d.N % 4 == 0 && d.a_splits >= 1 &&
           d.a_splits <= WSK_MAX_ASPLITS && d.a_slab_stride % 4 == 0 && aligned16(d.a_slab) && aligned16(d.a_bias) &&
           aligned16(d.a_out);
  if (d.b_kc) return d.epi == EPI_DX; // dX: B = W^T stored k-contiguous
  return d.N % 4 == 0 && (d.epi == EPI_FWD || d.epi == EPI_STORE || d.epi == EPI_HEAD);
}

template <bool AKC, bool BKC, int EPI> void dispatch_tile(hipStream_t s, const GemmDesc &d) {
  // LDS-DMA stages: as many tile buffers as fit two workgroups per CU (80 KB each); the register-staged
  // fallback (gathered mn-contiguous operands, odd shapes) keeps two k-tiles of loads in flight
  if (d.tile == TILE_32x128) {
    if constexpr (AKC) {
      if (wsk_ok(d)) { // the wave-split-K direct-load loop (gemm_wsk_kernel)
        GemmK k = make_gemmk<32, 128>(d);
        const dim3 grid(unsigned(k.gx), unsigned(k.gy), unsigned((d.splits > 1 ? d.splits : 1) + k.side_planes));
        if (d.a_slab) {
          if constexpr (!BKC && EPI != EPI_HEAD && EPI != EPI_DX)
            hipLaunchKernelGGL((gemm_wsk_kernel<EPI, false, false, true>), grid, dim3(256), 0, s, k);
        } else if (d.a_idx) {
          hipLaunchKernelGGL((gemm_wsk_kernel<EPI, true, BKC, false>), grid, dim3(256), 0, s, k);
        } else {
          hipLaunchKernelGGL((gemm_wsk_kernel<EPI, false, BKC, false>), grid, dim3(256), 0, s, k);
        }
        return;
      }
    }
    // 32 x 128 (20 KB per stage), one 8-wave workgroup (two k-groups) per CU: the LDS-DMA loop (A from the
    // previous layer's slabs, dX, shapes the direct loop does not take)
    launch<1, 4, 1, 1, AKC, BKC, EPI, 2, 2, 4>(s, d);
  } else if (d.tile == TILE_64x128) { // 64 x 128 (24 KB per stage), two workgroups per CU
    launch<2, 2, 1, 2, AKC, BKC, EPI, 1, 2, 3>(s, d);
  } else if (d.tile == TILE_64x64) { // 64 x 64 (16 KB per stage)
    launch<2, 2, 1, 1, AKC, BKC, EPI, 1, 2, 5>(s, d);
  } else if (d.N > 64) { // 128 x 128 (32 KB per stage)
    launch<2, 2, 2, 2, AKC, BKC, EPI, 1, 2, 2>(s, d);
  } else if (d.N > 32) launch<2, 2, 2, 1, AKC, BKC, EPI, 1, 1, 3>(s, d); // 128 x 64 (24 KB per stage)
  else launch<4, 1, 1, 1, AKC, BKC, EPI, 1, 1, 3>(s, d);                 // 128 x 32 (20 KB per stage)
}

} // namespace

void gemm_tile_for(int N, int tile, int *BM, int *BN) {
  if (tile == TILE_32x128) {
    *BM = 32;
    *BN = 128;
    return;
  }
  if (tile == TILE_64x64) {
    *BM = 64;
    *BN = 64;
    return;
  }
  if (tile == TILE_64x128) {
    *BM = 64;
    *BN = 128;
    return;
  }
  *BM = 128;
  *BN = N > 64 ? 128 : (N > 32 ? 64 : 32);
}

int gemm_row_tiles(int M, int tile) {
  int BM, BN;
  gemm_tile_for(128, tile, &BM, &BN);
  return (M + BM - 1) / BM;
}

long long gemm_tiles(const GemmDesc &d) {
  int BM, BN;
  gemm_tile_for(d.N, d.tile, &BM, &BN);
  return cdiv((long long)d.M, (long long)BM) * cdiv((long long)d.N, (long long)BN);
}

bool gemm_asum_ok(const GemmDesc &d) {
  const int kc = d.splits > 1 ? d.k_chunk : d.K;
  return d.tile == TILE_32x128 && d.a_kc && !d.b_kc && !d.a_idx && (d.epi == EPI_STORE || d.epi == EPI_FWD) &&
         d.K % 4 == 0 && d.lda % 4 == 0 && d.ldb % 4 == 0 && d.a_slab_stride % 4 == 0 && kc > 0 && kc <= 4 * 32 &&
         d.a_splits >= 1 && aligned16(d.A) && aligned16(d.B) && aligned16(d.a_slab) && aligned16(d.a_bias) &&
         aligned16(d.a_out);
}

static bool glds_fast(const GemmDesc &d) { // launch()'s FAST conditions for mn-contiguous A and B
  return d.K % 4 == 0 && d.lda % 4 == 0 && d.ldb % 4 == 0 && aligned16(d.A) && aligned16(d.B) &&
         (d.a_mvalid > 0 ? d.a_mvalid : d.M) % 4 == 0 && d.N % 4 == 0;
}

bool gemm_group_ok(const GemmDesc &d1, const GemmDesc &d2) {
  auto one = [](const GemmDesc &d) {
    return d.M > 0 && d.N > 0 && d.epi == EPI_STORE && !d.a_kc && !d.b_kc && d.tile == TILE_64x64 && !d.a_idx &&
           !d.a_slab && glds_fast(d);
  };
  return one(d1) && one(d2) && !(d2.side_slab && d2.side_count > 0);
}

void gemm_group(hipStream_t s, const GemmDesc &d1, const GemmDesc &d2) {
  if (!gemm_group_ok(d1, d2)) throw std::runtime_error("gemm_group: two 64 x 64 mn-contiguous split-K GEMMs");
  launch<2, 2, 1, 1, false, false, EPI_STORE, 1, 2, 5>(s, d1, &d2); // dispatch_tile's TILE_64x64 instance
  LBF_KERNEL_CHECK();
}

void gemm(hipStream_t s, const GemmDesc &d) {
  if (d.M <= 0 || d.N <= 0) return;
  if (d.a_slab && !gemm_asum_ok(d)) throw std::runtime_error("gemm: A from slabs not supported for this shape");
  if (d.epi == EPI_HEAD) {
    int BM, BN;
    gemm_tile_for(d.N, d.tile, &BM, &BN);
    if (!(d.a_kc && !d.b_kc) || d.N > BN || d.splits > 1 || d.head_out < 1 || d.head_out > headc::HMAX_OUT)
      throw std::runtime_error("gemm: EPI_HEAD needs an unsplit forward GEMM with N <= the tile width");
    if (d.head_fold >= 0 &&
        (d.N > 128 || d.head_fold > headc::FOLD_MAX || d.head_fold % 4 || d.head_fold_c0 % 4 || d.lda % 4 ||
         d.head_fold_c0 + d.head_fold != d.K || !aligned16(d.A)))
      throw std::runtime_error("gemm: EPI_HEAD fold needs N <= 128, <= 16 aligned input columns ending at K");
    dispatch_tile<true, false, EPI_HEAD>(s, d);
  } else if (d.epi == EPI_FWD && d.a_kc && !d.b_kc) dispatch_tile<true, false, EPI_FWD>(s, d);
  else if (d.epi == EPI_DX && d.a_kc && d.b_kc) dispatch_tile<true, true, EPI_DX>(s, d);
  else if (d.epi == EPI_STORE && !d.a_kc && !d.b_kc) dispatch_tile<false, false, EPI_STORE>(s, d);
  else if (d.epi == EPI_STORE && d.a_kc && !d.b_kc) dispatch_tile<true, false, EPI_STORE>(s, d);
  else throw std::runtime_error("gemm: unsupported operand/epilogue combination");
  LBF_KERNEL_CHECK();
}

} // namespace lbf

#ifdef LBF_KTRACE
extern "C" int lbf_dbg_ktrace_gemm(unsigned long long *host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(lbf::lbf_kt_buf), size_t(n) * 8) == hipSuccess ? 0 : 1;
}
extern "C" int lbf_dbg_ktrace_gemm_blk(unsigned long long *host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(lbf::lbf_kt_blk), sizeof(lbf::lbf_kt_blk)) == hipSuccess ? 0 : 1;
}
extern "C" int lbf_dbg_ktrace_gemm_hw(unsigned long long *host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(lbf::lbf_kt_hw), sizeof(lbf::lbf_kt_hw)) == hipSuccess ? 0 : 1;
}
#endif
