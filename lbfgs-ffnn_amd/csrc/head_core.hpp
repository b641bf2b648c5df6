// Output layer ("head") for Out <= 16 outputs on a hidden width H <= 256, on one 64-sample tile of
// activations in LDS. Shared by the standalone head kernel (head.hip: tiles streamed from HBM) and
// the forward GEMM's EPI_HEAD epilogue (gemm.hip: the tile comes straight from the accumulators, so
// the last hidden layer's activations never go to HBM).
//
// From one LDS copy of the tile's activations A[b][0..H) it runs the three small products of the last
// layer on MFMA (v_mfma_f32_16x16x4_f32, Out padded to 16):
//   forward  Z = A W + b ; a = act(Z) ; d = a - y ; sse += d^2 ; dZ = d * act'(a) * inv_scale
//   delta    D = (dZ W^T) .* act_prev'(A)                        -> global, feeds the next dW GEMM
//   weights  [dW ; db] += [A | 1]^T dZ                             (accumulators stay in registers)
// Replaces for the last layer the reference's forward Sgemm + add_bias + activation, diff_kernel +
// Sdot + Sscal, activation_deriv + dW Sgemm + sum_rows + dX Sgemm (src/cuda/layer.cuh:48-105,
// src/cuda/network.cuh:97-119, src/cuda/kernels.cuh:74-153).
//
// 16x16x4 f32 MFMA: lane l feeds A[l&15][k = l>>4] and B[k = l>>4][l&15]; accumulator r of lane l is
// C[(l>>4)*4 + r][l&15]. Within a K-run of 4S values, lane group g = l>>4 consumes k = g*S + s at
// step s (a permutation of the summation order), so k-contiguous operands are ds_read_b128 runs.
// Block: 4 working waves; wave w < 4 owns samples 16w..16w+15 of the tile. Larger blocks (the GEMM's
// 8-wave variant) join the barriers and the cooperative copies only.
#pragma once

#include "act.hpp"
#include "internal.hpp"
#include "kernels.hpp"
#include "wave.hpp"

#include <hip/hip_runtime.h>

namespace lbf {

namespace headc {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int HMAX = 256;
constexpr int HMAX_OUT = 16;
constexpr int TB = 64;                     // samples per tile (4 strips of 16, one per wave)
constexpr int LDZ = 20;                    // dZ row stride (16 + 4): conflict-free b128 rows
constexpr int QMAX = (HMAX + 1 + 63) / 64; // dW strips per wave: ceil(ceil((H+1)/16) / 4)
constexpr __host__ __device__ int qstrips(int H) { return (H + 1 + 63) / 64; }

__device__ __forceinline__ int round64(int x) { return (x + 63) & ~63; }

constexpr int XLD = 20;                    // folded input-column rows [yrows][XLD]: conflict-free b32 reads
constexpr int FOLD_MAX = 16;               // input columns a GEMM epilogue can fold (one 16-wide strip)

// Column order of the 16 (padded) outputs in Dz and Wr: output o sits at column ocol(o). A 16-B read of
// columns 4g..4g+3 then gives lane group g the outputs 4kk + g (kk = 0..3), so step kk of the delta product's
// MFMA chain consumes outputs 4kk .. 4kk+3 and the chain stops after ceil(Out / 4) steps (Out = 10: three of
// four; the skipped steps multiplied zeros).
__host__ __device__ constexpr int ocol(int o) { return (o & 3) * 4 + (o >> 2); }

// LDS carve-up (floats): As [TB][LDA] | Wt [16][LDA] | Wr [Hp][16] | Dz [TB][LDZ] | bias [16] | red [8]
// The GEMM epilogue appends hb [Hp] (the hidden layer's bias), ys [yrows][16] (the block's targets)
// and xr [yrows][XLD] (the input columns folded into the epilogue, see TileArgs::fold).
struct Smem {
  float *As, *Wt, *Wr, *Dz, *bias, *hb, *ys, *xr;
  double *red;
  int H, Hp, LDA;
};
constexpr __host__ __device__ int smem_floats(int H) {
  const int Hp = (H + 63) & ~63, LDA = Hp + 4;
  return TB * LDA + 16 * LDA + Hp * 16 + TB * LDZ + 16 + 8;
}
constexpr __host__ __device__ int smem_floats_epi(int H, int yrows) {
  return smem_floats(H) + ((H + 63) & ~63) + yrows * 16 + yrows * XLD;
}
__device__ inline Smem carve(float *base, int H) {
  Smem s;
  s.H = H;
  s.Hp = round64(H);
  s.LDA = s.Hp + 4;
  s.As = base;
  s.Wt = s.As + TB * s.LDA;
  s.Wr = s.Wt + 16 * s.LDA;
  s.Dz = s.Wr + s.Hp * 16;
  s.bias = s.Dz + TB * LDZ;
  s.red = reinterpret_cast<double *>(s.bias + 16); // 8-byte aligned: every region above is a multiple of 2
  s.hb = s.bias + 16 + 8;                           // after red (4 doubles)
  s.ys = s.hb + s.Hp;
  s.xr = nullptr; // the GEMM epilogue sets it (after its ys rows)
  return s;
}

// W (both orientations) and the bias into LDS. Block-wide; ends with __syncthreads.
__device__ inline void stage_w(const Smem &s, const float *P, int Out) {
  const int t = threadIdx.x, nt = blockDim.x;
  for (int e = t; e < 16 * s.LDA; e += nt) s.Wt[e] = 0.0f;
  for (int e = t; e < s.Hp * 16; e += nt) s.Wr[e] = 0.0f;
  __syncthreads();
  for (int e = t; e < s.H * Out; e += nt) {
    const int i = e / Out, o = e - i * Out;
    const float v = P[e];
    s.Wt[o * s.LDA + i] = v;
    s.Wr[i * 16 + ocol(o)] = v;
  }
  if (t < HMAX_OUT) s.bias[t] = t < Out ? P[(long long)s.H * Out + t] : 0.0f;
  __syncthreads();
}

// Everything the GEMM epilogue reads from HBM, loaded into registers in one batch (issued before the
// block's last k-tile is computed, so the latency hides behind it) and written to LDS afterwards:
// W as Wt/Wr (every element of [16][Hp] written once, zeros outside Out x H), both biases and the
// block's target rows. HN: the tile width (>= Hp), YR: the tile's rows, NT: threads in the block.
template <int HN, int YR, int NT>
struct EpiPrefetch {
  static constexpr int PW = (16 * HN + NT - 1) / NT, PY = (YR * 16 + NT - 1) / NT;
  static constexpr int PX = (YR * 4 + NT - 1) / NT; // 16-B chunks of the folded input columns
  static_assert(NT >= HN + 16, "one thread per bias element");
  float w[PW], y[PY], hb, ob;
  f32x4 x[PX];

  // The block's rows of the folded input columns [c0, c0 + nfold) (nfold % 4 == 0, 16-B aligned rows):
  // unconditional loads from clamped addresses, masked afterwards.
  __device__ inline void load_fold(const float *A, long long lda, const int *aidx, int c0, int nfold, long long m0,
                                   long long M) {
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < PX; ++j) {
      const int e = t + j * NT, r = e >> 2, q = e & 3;
      const bool ok = e < YR * 4 && 4 * q < nfold && m0 + r < M;
      const long long m = ok ? m0 + r : 0;
      const long long row = aidx ? (long long)aidx[m] : m;
      const f32x4 v = *reinterpret_cast<const f32x4 *>(A + row * lda + c0 + (ok ? 4 * q : 0));
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      const unsigned k = ok ? 0xffffffffu : 0u;
      x[j] = __builtin_bit_cast(f32x4, __builtin_bit_cast(u32x4, v) & (u32x4){k, k, k, k});
    }
  }
  __device__ inline void store_fold(const Smem &s) const {
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < PX; ++j) {
      const int e = t + j * NT;
      if (e < YR * 4) *reinterpret_cast<f32x4 *>(s.xr + (e >> 2) * XLD + 4 * (e & 3)) = x[j];
    }
  }

  __device__ inline void load(const float *P, int H, int Out, const float *bias, const float *Y, const int *idx,
                              long long m0, long long M) {
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < PW; ++j) {
      const int e = t + j * NT, o = e / HN, i = e % HN;
      w[j] = (e < 16 * HN && o < Out && i < H) ? P[i * Out + o] : 0.0f;
    }
    hb = t < H ? bias[t] : 0.0f;
    ob = (t >= HN && t < HN + Out) ? P[(long long)H * Out + (t - HN)] : 0.0f;
#pragma unroll
    for (int j = 0; j < PY; ++j) {
      const int e = t + j * NT, r = e >> 4, o = e & 15;
      const long long m = m0 + r;
      float v = 0.0f;
      if (e < YR * 16 && o < Out && m < M) v = Y[(idx ? (long long)idx[m] : m) * Out + o];
      y[j] = v;
    }
  }
  __device__ inline void store(const Smem &s) const {
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < PW; ++j) {
      const int e = t + j * NT, o = e / HN, i = e % HN;
      if (e < 16 * HN && i < s.Hp) {
        s.Wt[o * s.LDA + i] = w[j];
        s.Wr[i * 16 + ocol(o)] = w[j];
      }
    }
    if (t < s.Hp) s.hb[t] = hb;
    if (t >= HN && t < HN + 16) s.bias[t - HN] = ob;
#pragma unroll
    for (int j = 0; j < PY; ++j) {
      const int e = t + j * NT;
      if (e < YR * 16) s.ys[e] = y[j];
    }
  }
};

struct TileArgs {
  const float *Y;
  const int *idx;
  const float *ys; // LDS targets [TB][16] of this tile (GEMM epilogue) or null: Y / idx from global
  int Out, act_out, act_prev;
  float sc; // inv_scale
  float *delta;
  bool vec; // 16-B aligned rows (the standalone kernel's staging loads)
  // Fold (GEMM epilogue, H <= 128): the rows of the previous layer's [dW ; db] that its dW GEMM's
  // last, mostly empty row tile would hold — input columns c0 .. c0+nfold-1 and the bias row — are
  // accumulated here from the delta accumulators: fold[i][c] += sum_b x[b][c0+i] delta[b][c] and
  // db[c] += sum_b delta[b][c]. xr: this tile's rows of those input columns in LDS ([TB][XLD]).
  const float *xr;
  int nfold;
};
// Per-lane fold accumulators: wave w owns the delta columns of strips 2w and 2w+1.
struct FoldAcc {
  f32x4 c[2];
  float db[2];
};
// The part of the hidden width one workgroup covers (the standalone head splits H over workgroups when a
// batch has few tiles; the forward Z is then computed by each of them): [dW ; db] row strips [st0, st1)
// (strip = 16 rows, the bias row included in the last) and delta column strips [cb0, cb1) (cb0 even).
// Default: everything.
struct HRange {
  int st0 = 0, st1 = 1 << 20, cb0 = 0, cb1 = 1 << 20;
};

// One tile: s.As holds the activations of samples b0..b0+rows-1 (zero-padded to Hp columns), staged
// and followed by a barrier. Accumulates [dW ; db] into cw and the SSE into sse; writes the tile's
// delta rows to global straight from the MFMA accumulators. Ends with an LDS barrier (As free again).
// QM: dW strips per wave (>= ceil(ceil((H+1)/16)/4)); strips past H are skipped (wave-uniform).
// Barriers here only order LDS (lds_barrier): a __syncthreads would also wait for the delta stores.
// FOLD: accumulate the fold (TileArgs::xr / nfold) into fa; needs H <= 128 (one pass of column strips).
// TBR: samples the tile holds (64, or 32 for a 32-row GEMM tile: the products over samples then run half
// their steps; rows >= TBR of As / Dz / ys / xr are neither read nor needed).
template <bool EXTRA_WAVES, int QM, bool FOLD, int TBR = TB> // EXTRA_WAVES: waves >= 4 only join barriers
__device__ inline void tile(const Smem &s, const TileArgs &a, long long b0, int rows, f32x4 (&cw)[QM], double &sse,
                            FoldAcc &fa, const HRange &hr = HRange()) {
  static_assert(TBR == 64 || TBR == 32, "head tile of 64 or 32 samples");
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int r0 = wave * 16, LDA = s.LDA, H = s.H;
  const bool active = !EXTRA_WAVES || wave < 4;
  const bool zrows = active && wave < TBR / 16; // wave-uniform: this wave's 16 samples are in the tile
  const int dzc = ocol(li);                      // this lane's output column in Dz (see ocol)
  KT(34);
  // ---- forward: Z strip (16 samples x 16 outputs) of this wave, two interleaved chains ----
  f32x4 acc = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  for (int kc = 0; zrows && kc < s.Hp; kc += 32) { // 32 k per round: 8 steps, two chains
    float af[8], bf[8];
    const int kh = kc & 63, k64 = kc & ~63; // lane group g consumes k = k64 + 16 g + s, s = kh/4 .. kh/4 + 7
    const float *pa = s.As + (r0 + li) * LDA + k64 + g * 16 + (kh >> 2);
    const float *pb = s.Wt + li * LDA + k64 + g * 16 + (kh >> 2);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const f32x4 va = *reinterpret_cast<const f32x4 *>(pa + 4 * q);
      const f32x4 vb = *reinterpret_cast<const f32x4 *>(pb + 4 * q);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        af[4 * q + j] = va[j];
        bf[4 * q + j] = vb[j];
      }
    }
#pragma unroll
    for (int st = 0; st < 8; st += 2) {
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(af[st], bf[st], acc, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(af[st + 1], bf[st + 1], acc1, 0, 0, 0);
    }
  }
  acc += acc1;
  KT(35);
  // ---- loss and dZ (lane: samples r0 + g*4 + r, output o = li); targets loaded as one batch ----
  if (zrows) {
    float yv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + g * 4 + r;
      yv[r] = 0.0f;
      if (row < rows && li < a.Out) {
        if (a.ys) yv[r] = a.ys[row * 16 + li];
        else yv[r] = a.Y[(a.idx ? (long long)a.idx[b0 + row] : b0 + row) * a.Out + li];
      }
    }
    with_act(a.act_out, [&](auto AC) __attribute__((always_inline)) {
      constexpr int A = decltype(AC)::value;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + g * 4 + r;
        float dz = 0.0f;
        if (row < rows && li < a.Out) {
          const float av = act_c<A>(acc[r] + s.bias[li]);
          const float d = av - yv[r];
          sse += double(d) * double(d);
          dz = d * dact_c<A>(av) * a.sc;
        }
        s.Dz[row * LDZ + dzc] = dz;
      }
    });
  }
  lds_barrier();
  KT(36);
  // ---- [dW ; db] += [A | 1]^T dZ over this tile (strips of 16 rows i; row H is the bias) ----
  // Step k of lane group g takes sample b = (k & 3) + 4g + 16(k >> 2): the four groups of a step read
  // rows 4 apart (bank offset 16 with LDA = 4 mod 64, 80 with LDZ = 20), so the reads are
  // conflict-free. Every LDS read is unconditional (clamped column) and all are issued before the
  // MFMA chains; strips past the bias row are skipped wave-uniformly. A strip holding only the bias row
  // (H % 16 == 0) is a column sum of dZ on the VALU: sixteen MFMAs for one useful row otherwise.
  if (active) {
#pragma unroll
    for (int q = 0; q < QM; ++q) {
      const int st = hr.st0 + wave + 4 * q;
      if (st * 16 > H || st >= hr.st1) continue; // wave-uniform
      if (st * 16 == H) { // db[o] += sum_b dZ[b][o]: lane group g sums samples b = g mod 4, then the groups
        float d = 0.0f;
#pragma unroll
        for (int b = 0; b < TBR; b += 4) d += s.Dz[(b + g) * LDZ + dzc];
        d += __shfl_xor(d, 16);
        d += __shfl_xor(d, 32);
        if (g == 0) cw[q][0] += d;
        continue;
      }
      const int ic = st * 16 + li;
      const int icc = ic < H ? ic : 0;
      const bool bias_strip = st * 16 + 15 >= H; // wave-uniform
      f32x4 c = cw[q];
#pragma unroll 1
      for (int k0 = 0; k0 < TBR / 4; k0 += 4) { // four steps of loads in flight, then their MFMAs
        float av[4], dz[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int b = k + 4 * g + k0 * 4; // (k & 3) + 4g + 16 (k >> 2) for step k0 + k
          dz[k] = s.Dz[b * LDZ + dzc];
          av[k] = s.As[b * LDA + icc];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float x = bias_strip ? (ic < H ? av[k] : (ic == H ? 1.0f : 0.0f)) : av[k];
          c = __builtin_amdgcn_mfma_f32_16x16x4f32(x, dz[k], c, 0, 0, 0);
        }
      }
      cw[q] = c;
    }
  }
  KT(37);
  // ---- delta = (dZ W^T) .* act_prev'(A), stored from the accumulators ----
  // Wave w takes the column strips 2w, 2w+1 (+8, +9, ... for H > 128) over all TB rows, one 16-row
  // strip at a time (two MFMA chains of 4 each). Lanes li of a row write 64 contiguous bytes.
  // Strip cb+1 may pass H: Wr's zero rows (Hp >= 16 (cb + 2)) make it zero and nothing is stored.
  // The k = output dimension runs ceil(Out / 4) MFMA steps (Dz / Wr column order ocol).
  if (a.delta && active) {
    const int ncs = (H + 15) >> 4;
    const int nks = (a.Out + 3) >> 2; // uniform
    with_act(a.act_prev, [&](auto AC) __attribute__((always_inline)) {
      constexpr int A = decltype(AC)::value;
      for (int cb = hr.cb0 + 2 * wave; cb < ncs && cb < hr.cb1; cb += 8) { // wave-uniform; one pass when H <= 128
        const f32x4 wb0 = *reinterpret_cast<const f32x4 *>(s.Wr + (cb * 16 + li) * 16 + g * 4);
        const f32x4 wb1 = *reinterpret_cast<const f32x4 *>(s.Wr + ((cb + 1) * 16 + li) * 16 + g * 4);
        const int col = cb * 16 + li;
#pragma unroll 1
        for (int rs = 0; rs < TBR / 16; ++rs) {
          const f32x4 da = *reinterpret_cast<const f32x4 *>(s.Dz + (rs * 16 + li) * LDZ + g * 4);
          float ap0[4], ap1[4], xa[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) { // columns < 16 (cb + 2) <= Hp: always inside the row
            const float *p = s.As + (rs * 16 + g * 4 + r) * LDA + col;
            ap0[r] = p[0];
            ap1[r] = p[16];
            if constexpr (FOLD) xa[r] = a.xr[(rs * 16 + g * 4 + r) * XLD + li];
          }
          f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (k < nks) { // uniform
              c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(da[k], wb0[k], c0, 0, 0, 0);
              c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(da[k], wb1[k], c1, 0, 0, 0);
            }
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = rs * 16 + g * 4 + r;
            const float d0 = c0[r] * dact_c<A>(ap0[r]);
            const float d1 = c1[r] * dact_c<A>(ap1[r]);
            if (row < rows) {
              float *d = a.delta + (b0 + row) * H + col;
              if (col < H) d[0] = d0;
              if (col + 16 < H) d[16] = d1;
            }
            if constexpr (FOLD) { // rows past `rows` have dZ = 0, so d0 = d1 = 0 there
              // B operand: lane (li, g) holds delta[row(k = g)][column li]; A operand: x[row(k = g)][i = li]
              fa.c[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[r], d0, fa.c[0], 0, 0, 0);
              fa.c[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[r], d1, fa.c[1], 0, 0, 0);
              fa.db[0] += d0;
              fa.db[1] += d1;
            }
          }
        }
      }
    });
  }
  KT(38);
  lds_barrier(); // every wave done reading As / Dz
  KT(39);
}

// The fold's partial rows [nfold + 1][H] (input columns, then the bias row) of the workgroup's slab.
// Every lane runs the shuffles; H <= 128.
__device__ inline void write_fold(const FoldAcc &fa, int H, int nfold, float *slab) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int li = lane & 15, g = lane >> 4;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    float db = fa.db[j];
    db += __shfl_xor(db, 16); // sum over the four row groups, fixed order
    db += __shfl_xor(db, 32);
    const int col = (2 * wave + j) * 16 + li;
    if (wave < 4 && col < H) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (g * 4 + r < nfold) slab[(g * 4 + r) * H + col] = fa.c[j][r];
      if (g == 0) slab[nfold * H + col] = db;
    }
  }
}

// The workgroup's [dW ; db] partial slab and SSE partial.
// With an HRange narrower than the whole width, the slab's rows outside [16 st0, 16 st1) are written as
// zeros (a sibling workgroup owns them), so the fixed-order slab reduction stays bitwise the same.
template <int QM>
__device__ inline void write_partials(const Smem &s, int Out, const f32x4 (&cw)[QM], double sse, float *slab,
                                      double *sse_out, const HRange &hr = HRange()) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int li = lane & 15, g = lane >> 4, H = s.H;
  if (hr.st0 > 0 || hr.st1 * 16 < H + 1)
    for (int e = t; e < (H + 1) * Out; e += blockDim.x) {
      const int row = e / Out;
      if (row < hr.st0 * 16 || row >= hr.st1 * 16) slab[e] = 0.0f;
    }
  if (wave < 4 && li < Out) {
#pragma unroll
    for (int q = 0; q < QM; ++q) {
      const int st = hr.st0 + wave + 4 * q;
      if (st * 16 < H + 1 && st < hr.st1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = st * 16 + g * 4 + r;
          if (i <= H) slab[i * Out + li] = cw[q][r];
        }
      }
    }
  }
  sse = wave_sum_f64(sse);
  if (lane == 0 && wave < 4) s.red[wave] = sse;
  lds_barrier();
  if (t == 0) *sse_out = ((s.red[0] + s.red[1]) + s.red[2]) + s.red[3];
}

} // namespace headc

} // namespace lbf
