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
#include "kernels.hpp"
#include "wave.hpp"

#include <hip/hip_runtime.h>

namespace lbf {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float h_act(int a, float x) {
  switch (a) {
  case ACT_TANH: return tanhf(x);
  case ACT_RELU: return x > 0.0f ? x : 0.0f;
  case ACT_SIGMOID: return 1.0f / (1.0f + expf(-x));
  default: return x;
  }
}
__device__ __forceinline__ float h_dact(int a, float y) {
  switch (a) {
  case ACT_TANH: return 1.0f - y * y;
  case ACT_RELU: return y > 0.0f ? 1.0f : 0.0f;
  case ACT_SIGMOID: return y * (1.0f - y);
  default: return 1.0f;
  }
}

__device__ __forceinline__ double h_wave_sum(double v) { return wave_sum_f64(v); }

constexpr int HMAX = 256;
constexpr int HMAX_OUT = 16;
constexpr int TB = 64;                         // samples per tile (4 strips of 16, one per wave)
constexpr int LDZ = 20;                        // dZ row stride (16 + 4): conflict-free b128 rows
constexpr int QMAX = (HMAX + 1 + 63) / 64;     // dW strips per wave: ceil(ceil((H+1)/16) / 4)
constexpr int MAX_WG = 512;                    // 2 workgroups per CU

__device__ __forceinline__ int round64(int x) { return (x + 63) & ~63; }

__global__ __launch_bounds__(256) void head_kernel(const float *A, int H, const float *P, int Out, const float *Y,
                                                   const int *idx, long long B, int act_out, int act_prev,
                                                   double inv_scale, float *delta, float *slab, double *sse_part,
                                                   const int *abort) {
  if (abort && *abort) return;
  extern __shared__ __attribute__((aligned(16))) float sh[];
  const int Hp = round64(H);
  const int LDA = Hp + 4;
  float *As = sh;                  // [TB][LDA]   activations (zero-padded to Hp), then delta in place
  float *Wt = As + TB * LDA;       // [16][LDA]   Wt[o][i] = W[i][o]
  float *Wr = Wt + 16 * LDA;       // [Hp][16]    Wr[i][o] = W[i][o]
  float *Dz = Wr + Hp * 16;        // [TB][LDZ]
  __shared__ float bias_s[HMAX_OUT];
  __shared__ double red[4];

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int li = lane & 15, g = lane >> 4;
  const long long ntiles = (B + TB - 1) / TB;
  const bool vec = (H & 3) == 0 && ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(delta)) & 15) == 0;
  const int Hq = H >> 2;

  // ---- stage W (both orientations) and the bias once ----
  for (int e = t; e < 16 * LDA; e += 256) Wt[e] = 0.0f;
  for (int e = t; e < Hp * 16; e += 256) Wr[e] = 0.0f;
  __syncthreads();
  for (int e = t; e < H * Out; e += 256) {
    const int i = e / Out, o = e - i * Out;
    const float v = P[e];
    Wt[o * LDA + i] = v;
    Wr[i * 16 + o] = v;
  }
  if (t < HMAX_OUT) bias_s[t] = t < Out ? P[(long long)H * Out + t] : 0.0f;

  f32x4 cw[QMAX];
#pragma unroll
  for (int q = 0; q < QMAX; ++q) cw[q] = (f32x4){0.f, 0.f, 0.f, 0.f};
  double sse = 0.0;
  const float sc = float(inv_scale);
  const int r0 = wave * 16;

  for (long long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const long long b0 = tile * TB;
    const int rows = int(min((long long)TB, B - b0));
    __syncthreads(); // previous tile's delta store done with As
    // ---- stage the activation tile ----
    if (vec) {
      for (int e = t; e < TB * (Hp >> 2); e += 256) {
        const int r = e / (Hp >> 2), c4 = e - r * (Hp >> 2);
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (r < rows && c4 < Hq) v = *reinterpret_cast<const f32x4 *>(A + (b0 + r) * H + 4 * c4);
        *reinterpret_cast<f32x4 *>(As + r * LDA + 4 * c4) = v;
      }
    } else {
      for (int e = t; e < TB * Hp; e += 256) {
        const int r = e / Hp, c = e - r * Hp;
        As[r * LDA + c] = (r < rows && c < H) ? A[(b0 + r) * H + c] : 0.0f;
      }
    }
    __syncthreads();

    // ---- forward: Z strip (16 samples x 16 outputs) of this wave ----
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int kc = 0; kc < Hp; kc += 64) {
      float af[16], bf[16];
      const float *pa = As + (r0 + li) * LDA + kc + g * 16;
      const float *pb = Wt + li * LDA + kc + g * 16;
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
      for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(af[s], bf[s], acc, 0, 0, 0);
    }
    // ---- loss and dZ (lane: samples r0 + g*4 + r, output o = li) ----
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + g * 4 + r;
      float dz = 0.0f;
      if (row < rows && li < Out) {
        const float a = h_act(act_out, acc[r] + bias_s[li]);
        const long long yr = idx ? (long long)idx[b0 + row] : b0 + row;
        const float d = a - Y[yr * Out + li];
        sse += double(d) * double(d);
        dz = d * h_dact(act_out, a) * sc;
      }
      Dz[row * LDZ + li] = dz;
    }
    __syncthreads();

    // ---- [dW ; db] += [A | 1]^T dZ over this tile (strips of 16 rows i; row H is the bias) ----
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
      const int st = wave + 4 * q;
      if (st * 16 < H + 1) {
        const int ic = st * 16 + li;
        f32x4 c = cw[q];
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const int b = g * 16 + s;
          const float a = ic < H ? As[b * LDA + ic] : (ic == H ? 1.0f : 0.0f);
          c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, Dz[b * LDZ + li], c, 0, 0, 0);
        }
        cw[q] = c;
      }
    }
    __syncthreads(); // every wave done reading As before delta overwrites it

    // ---- delta = (dZ W^T) .* act_prev'(A), in place over this wave's 16 rows ----
    if (delta) {
      const f32x4 da = *reinterpret_cast<const f32x4 *>(Dz + (r0 + li) * LDZ + g * 4);
      for (int it = 0; it * 16 < H; ++it) {
        const f32x4 wb = *reinterpret_cast<const f32x4 *>(Wr + (it * 16 + li) * 16 + g * 4);
        f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) c = __builtin_amdgcn_mfma_f32_16x16x4f32(da[s], wb[s], c, 0, 0, 0);
        const int i = it * 16 + li;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float *p = As + (r0 + g * 4 + r) * LDA + i;
          *p = c[r] * h_dact(act_prev, *p);
        }
      }
      __syncthreads();
      if (vec) {
        for (int e = t; e < rows * Hq; e += 256) {
          const int r = e / Hq, c4 = e - r * Hq;
          *reinterpret_cast<f32x4 *>(delta + (b0 + r) * H + 4 * c4) =
              *reinterpret_cast<const f32x4 *>(As + r * LDA + 4 * c4);
        }
      } else {
        for (int e = t; e < rows * H; e += 256) {
          const int r = e / H, c = e - r * H;
          delta[(b0 + r) * H + c] = As[r * LDA + c];
        }
      }
    }
  }

  // ---- this workgroup's [dW ; db] partial ----
  float *sl = slab + (long long)blockIdx.x * (H + 1) * Out;
  if (li < Out) {
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
      const int st = wave + 4 * q;
      if (st * 16 < H + 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = st * 16 + g * 4 + r;
          if (i <= H) sl[i * Out + li] = cw[q][r];
        }
      }
    }
  }
  sse = h_wave_sum(sse);
  if (lane == 0) red[wave] = sse;
  __syncthreads();
  if (t == 0) sse_part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

} // namespace

bool head_supported(int H, int Out) { return Out >= 1 && Out <= HMAX_OUT && H >= 1 && H <= HMAX; }
int head_tile(int) { return TB; }
// Workgroups (== partial slabs): one per tile up to MAX_WG, then a balanced number of tiles each.
int head_nwg(long long B, int) {
  const long long nt = cdiv(std::max(1LL, B), TB);
  if (nt <= MAX_WG) return int(nt);
  const long long per = cdiv(nt, MAX_WG);
  return int(cdiv(nt, per));
}

void head_fused(hipStream_t s, const float *A, int H, const float *P, int Out, const float *Y, const int *idx,
                long long B, int act_out, int act_prev, double inv_scale, float *delta, float *slab,
                double *sse_part, const int *abort) {
  const int Hp = (H + 63) & ~63;
  const size_t shmem = (size_t(TB) * (Hp + 4) + size_t(16) * (Hp + 4) + size_t(Hp) * 16 + size_t(TB) * LDZ) *
                       sizeof(float);
  static bool set = false;
  if (!set) {
    LBF_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(head_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 2048));
    set = true;
  }
  hipLaunchKernelGGL(head_kernel, dim3(head_nwg(B, H)), dim3(256), shmem, s, A, H, P, Out, Y, idx, B, act_out,
                     act_prev, inv_scale, delta, slab, sse_part, abort);
  LBF_KERNEL_CHECK();
}

} // namespace lbf
