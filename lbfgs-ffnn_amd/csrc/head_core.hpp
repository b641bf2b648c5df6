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

// LDS carve-up (floats): As [TB][LDA] | Wt [16][LDA] | Wr [Hp][16] | Dz [TB][LDZ] | bias [16] | red [8]
// The GEMM epilogue appends hb [Hp] (the hidden layer's bias) and ys [yrows][16] (the block's targets).
struct Smem {
  float *As, *Wt, *Wr, *Dz, *bias, *hb, *ys;
  double *red;
  int H, Hp, LDA;
};
constexpr __host__ __device__ int smem_floats(int H) {
  const int Hp = (H + 63) & ~63, LDA = Hp + 4;
  return TB * LDA + 16 * LDA + Hp * 16 + TB * LDZ + 16 + 8;
}
constexpr __host__ __device__ int smem_floats_epi(int H, int yrows) {
  return smem_floats(H) + ((H + 63) & ~63) + yrows * 16;
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
    s.Wr[i * 16 + o] = v;
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
  static_assert(NT >= HN + 16, "one thread per bias element");
  float w[PW], y[PY], hb, ob;

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
        s.Wr[i * 16 + o] = w[j];
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
  bool vec; // 16-B aligned delta rows
};

// One tile: s.As holds the activations of samples b0..b0+rows-1 (zero-padded to Hp columns), staged
// and followed by a __syncthreads. Accumulates [dW ; db] into cw and the SSE into sse; writes the
// tile's delta rows to global. Ends with __syncthreads (As free again).
// QM: dW strips per wave (>= ceil(ceil((H+1)/16)/4)); strips past H are computed and never written.
template <bool EXTRA_WAVES, int QM> // EXTRA_WAVES: blocks with more than 4 waves; waves >= 4 only join barriers
__device__ inline void tile(const Smem &s, const TileArgs &a, long long b0, int rows, f32x4 (&cw)[QM], double &sse) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int r0 = wave * 16, LDA = s.LDA, H = s.H;
  const bool active = !EXTRA_WAVES || wave < 4;
  KT(34);
  // ---- forward: Z strip (16 samples x 16 outputs) of this wave ----
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int kc = 0; active && kc < s.Hp; kc += 64) {
    float af[16], bf[16];
    const float *pa = s.As + (r0 + li) * LDA + kc + g * 16;
    const float *pb = s.Wt + li * LDA + kc + g * 16;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 va = *reinterpret_cast<const f32x4 *>(pa + 4 * q);
      const f32x4 vb = *reinterpret_cast<const f32x4 *>(pb + 4 * q);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        af[4 * q + j] = va[j];
        bf[4 * q + j] = vb[j];
      }
    }
#pragma unroll
    for (int st = 0; st < 16; ++st) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(af[st], bf[st], acc, 0, 0, 0);
  }
  KT(35);
  // ---- loss and dZ (lane: samples r0 + g*4 + r, output o = li); targets loaded as one batch ----
  if (active) {
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
        s.Dz[row * LDZ + li] = dz;
      }
    });
  }
  __syncthreads();
  KT(36);
  // ---- [dW ; db] += [A | 1]^T dZ over this tile (strips of 16 rows i; row H is the bias) ----
  // The QM strips are independent accumulation chains, interleaved per k.
  if (active) {
    f32x4 c[QM];
#pragma unroll
    for (int q = 0; q < QM; ++q) c[q] = cw[q];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int b = g * 16 + k;
      const float dz = s.Dz[b * LDZ + li];
#pragma unroll
      for (int q = 0; q < QM; ++q) {
        const int ic = (wave + 4 * q) * 16 + li;
        const float av = ic < H ? s.As[b * LDA + ic] : (ic == H ? 1.0f : 0.0f);
        c[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, dz, c[q], 0, 0, 0);
      }
    }
#pragma unroll
    for (int q = 0; q < QM; ++q) cw[q] = c[q];
  }
  __syncthreads(); // every wave done reading As before delta overwrites it
  KT(37);
  // ---- delta = (dZ W^T) .* act_prev'(A), in place over this wave's 16 rows, then stored ----
  // Column strips in pairs (two independent chains); strips past H read zero rows of Wr and write
  // only LDS padding.
  if (a.delta) {
    if (active) {
      const f32x4 da = *reinterpret_cast<const f32x4 *>(s.Dz + (r0 + li) * LDZ + g * 4);
      const int nit = ((H + 31) >> 5) << 1;
      with_act(a.act_prev, [&](auto AC) __attribute__((always_inline)) {
      constexpr int A = decltype(AC)::value;
      for (int it = 0; it < nit; it += 2) {
        const f32x4 wb0 = *reinterpret_cast<const f32x4 *>(s.Wr + (it * 16 + li) * 16 + g * 4);
        const f32x4 wb1 = *reinterpret_cast<const f32x4 *>(s.Wr + ((it + 1) * 16 + li) * 16 + g * 4);
        f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(da[k], wb0[k], c0, 0, 0, 0);
          c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(da[k], wb1[k], c1, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float *p = s.As + (r0 + g * 4 + r) * LDA + it * 16 + li;
          p[0] = c0[r] * dact_c<A>(p[0]);
          p[16] = c1[r] * dact_c<A>(p[16]);
        }
      }
      });
    }
    __syncthreads();
    KT(38);
    const int Hq = H >> 2, nt = blockDim.x;
    if (a.vec) {
      for (int e = t; e < rows * Hq; e += nt) {
        const int r = e / Hq, c4 = e - r * Hq;
        *reinterpret_cast<f32x4 *>(a.delta + (b0 + r) * H + 4 * c4) =
            *reinterpret_cast<const f32x4 *>(s.As + r * LDA + 4 * c4);
      }
    } else {
      for (int e = t; e < rows * H; e += nt) {
        const int r = e / H, c = e - r * H;
        a.delta[(b0 + r) * H + c] = s.As[r * LDA + c];
      }
    }
  }
  __syncthreads();
  KT(39);
}

// The workgroup's [dW ; db] partial slab and SSE partial.
template <int QM>
__device__ inline void write_partials(const Smem &s, int Out, const f32x4 (&cw)[QM], double sse, float *slab,
                                      double *sse_out) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int li = lane & 15, g = lane >> 4, H = s.H;
  if (wave < 4 && li < Out) {
#pragma unroll
    for (int q = 0; q < QM; ++q) {
      const int st = wave + 4 * q;
      if (st * 16 < H + 1) {
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
  __syncthreads();
  if (t == 0) *sse_out = ((s.red[0] + s.red[1]) + s.red[2]) + s.red[3];
}

} // namespace headc

} // namespace lbf
