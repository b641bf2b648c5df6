// Memory-bound kernels of the L-BFGS step (gfx950, wave64): the MSE output layer, split-K slab
// reduction, deterministic fp64 dot reductions, and the device-resident history (Gram sweep,
// coefficient two-loop, linear-combination sweep).
//
// Replaces: diff_kernel / sum_rows_kernel (src/cuda/kernels.cuh:136-153), cublasSdot / Snrm2 / Saxpy /
// Sscal with host pointer mode (kernels.cuh:28-50, every scalar a blocking device->host copy), and
// CudaLBFGS::compute_direction_ring (src/cuda/lbfgs.cuh:206-261, 2k+2 blocking dots + 2k axpys).
#include "act.hpp"
#include "internal.hpp"
#include "hist_core.hpp"
#include "kernels.hpp"
#include "wave.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>

namespace lbf {


typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------------------------
// wave / block reductions (fixed butterfly order -> bitwise reproducible)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) { return wave_sum_f64(v); }

// Sum NV values over a 256- or 512-thread block; result valid in thread 0. scratch: NV*16 doubles.
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double *scratch) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = wave_sum(v[i]);
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < NV; ++i) scratch[i * 16 + wave] = v[i];
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      double s = 0.0;
      for (int w = 0; w < nw; ++w) s += scratch[i * 16 + w];
      v[i] = s;
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------------------------
// reduce_rows: out[c] = sum_r P[r][c]   (one wave per column, lane-strided then butterfly)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void reduce_rows_kernel(const double *P, int nrows, int ncols, double *out) {
  const int col = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (col >= ncols) return;
  double s = 0.0;
  for (int r = lane; r < nrows; r += 64) s += P[(long long)r * ncols + col];
  s = wave_sum(s);
  if (lane == 0) out[col] = s;
}

void reduce_rows(hipStream_t s, const double *P, int nrows, int ncols, double *out) {
  if (ncols <= 0) return;
  hipLaunchKernelGGL(reduce_rows_kernel, dim3((ncols + 3) / 4), dim3(256), 0, s, P, nrows, ncols, out);
  LBF_KERNEL_CHECK();
}

// ---------------------------------------------------------------------------------------------
// fold_rows: out[j][c] = sum_{r in group j} P[r][c]; group j = rows [j*per, (j+1)*per). One block per
// (64-column group, row group): lane = column (coalesced 512-B row segments), wave w takes rows
// w, w+4, ... of the group, the four wave sums are added in a fixed order. Used to shrink a tall
// partial table (the Gram sweep's [nwg][6m+6] at large n) before a single-workgroup consumer.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fold_rows_kernel(const double *P, int nrows, int ncols, int per, double *out) {
  __shared__ double part[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int r0 = blockIdx.y * per, r1 = min(nrows, r0 + per);
  double s = 0.0;
  if (c < ncols) {
    for (int r = r0 + wave; r < r1; r += 4 * 8) { // eight independent loads in flight per lane
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = P[(long long)min(r + 4 * u, r1 - 1) * ncols + c]; // clamped: no per-load branch
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (r + 4 * u < r1) s += v[u];
    }
  }
  part[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && c < ncols)
    out[(long long)blockIdx.y * ncols + c] = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
}

int fold_rows(hipStream_t s, const double *P, int nrows, int ncols, int groups, double *out) {
  const int per = int(cdiv(nrows, groups));
  const int g = int(cdiv(nrows, per));
  hipLaunchKernelGGL(fold_rows_kernel, dim3(unsigned(cdiv(ncols, 64)), unsigned(g)), dim3(256), 0, s, P, nrows,
                     ncols, per, out);
  LBF_KERNEL_CHECK();
  return g;
}

// ---------------------------------------------------------------------------------------------
// Output layer: diff = A_out - Y ; dZ = diff * act'(A_out) * inv_scale ; partial sum(diff^2).
// src/cuda/network.cuh:97-107 (diff, 0.5*dot(diff,diff)/B, diff*=1/B) and layer.cuh:72 (act').
// ---------------------------------------------------------------------------------------------
int loss_partials_wg(long long B, int Out) {
  long long e = B * Out;
  long long w = cdiv(e, 256 * 8);
  return int(w < 1 ? 1 : (w > 1024 ? 1024 : w));
}

__global__ __launch_bounds__(256) void loss_diff_kernel(const float *A, long long lda, const float *Y, long long ldy,
                                                        const int *idx, long long B, int Out, int act,
                                                        double inv_scale, float *dZ, long long ldz,
                                                        double *partials) {
  __shared__ double scratch[16];
  const long long total = B * Out;
  const long long stride = (long long)gridDim.x * blockDim.x;
  double acc[1] = {0.0};
  const float sc = float(inv_scale);
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
    const long long b = e / Out;
    const int o = int(e - b * Out);
    const float a = A[b * lda + o];
    const long long yr = idx ? (long long)idx[b] : b;
    const float d = a - Y[yr * ldy + o];
    acc[0] += double(d) * double(d);
    dZ[b * ldz + o] = d * dact_rt(act, a) * sc;
  }
  block_sum<1>(acc, scratch);
  if (threadIdx.x == 0) partials[blockIdx.x] = acc[0];
}

void loss_diff(hipStream_t s, const float *Aout, long long lda, const float *Y, long long ldy, const int *idx,
               long long B, int Out, int act, double inv_scale, float *dZ, long long ldz, double *partials) {
  hipLaunchKernelGGL(loss_diff_kernel, dim3(loss_partials_wg(B, Out)), dim3(256), 0, s, Aout, lda, Y, ldy, idx, B,
                     Out, act, inv_scale, dZ, ldz, partials);
  LBF_KERNEL_CHECK();
}

// ---------------------------------------------------------------------------------------------
// split-K slab reduction -> flat gradient segment
// ---------------------------------------------------------------------------------------------
// Block = CW columns x (256/CW) split stripes; each thread sums its stripe, stripes combine in LDS in
// a fixed order. CW = 64 for few splits (coalesced 256-B rows), 16 when splits are many (more
// parallelism per column for the tall-and-thin slabs of small layers).
__global__ __launch_bounds__(256) void reduce_slabs_kernel(const float *slab, int splits, long long stride,
                                                           long long count, int cw, float *grad, const int *abort) {
  if (abort && *abort) return;
  __shared__ double part[256];
  const int t = threadIdx.x;
  const int nst = 256 / cw;
  const long long col = (long long)blockIdx.x * cw + (t % cw);
  const int stripe = t / cw;
  double s = 0.0;
  if (col < count)
    for (int k = stripe; k < splits; k += nst) s += double(slab[k * stride + col]);
  part[t] = s;
  __syncthreads();
  if (stripe == 0 && col < count) {
    double r = 0.0;
    for (int q = 0; q < nst; ++q) r += part[q * cw + t];
    grad[col] = float(r);
  }
}

__global__ __launch_bounds__(256) void fwd_reduce_act_kernel(const float *slab, int splits, long long stride, int M,
                                                             int N, const float *bias, int act, float *out,
                                                             const int *abort) {
  if (abort && *abort) return;
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)M * N) return;
  float v[8];
  float acc = 0.0f;
  int k = 0;
  for (; k + 8 <= splits; k += 8) { // independent loads in flight, summed in split order
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = slab[(long long)(k + u) * stride + e];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; k < splits; ++k) acc += slab[(long long)k * stride + e];
  const int n = int(e % N);
  const float z = acc + (bias ? bias[n] : 0.0f);
  out[e] = act_rt(act, z);
}

void fwd_reduce_act(hipStream_t s, const float *slab, int splits, long long stride, int M, int N, const float *bias,
                    int act, float *out, const int *abort) {
  const long long n = (long long)M * N;
  hipLaunchKernelGGL(fwd_reduce_act_kernel, dim3(unsigned(cdiv(n, 256))), dim3(256), 0, s, slab, splits, stride, M, N,
                     bias, act, out, abort);
  LBF_KERNEL_CHECK();
}

void reduce_slabs(hipStream_t s, const float *slab, int splits, long long stride, long long count, float *grad,
                  const int *abort) {
  const int cw = splits > 64 ? 16 : 64;
  hipLaunchKernelGGL(reduce_slabs_kernel, dim3(unsigned(cdiv(count, cw))), dim3(256), 0, s, slab, splits, stride,
                     count, cw, grad, abort);
  LBF_KERNEL_CHECK();
}

// ---------------------------------------------------------------------------------------------
// reduce_all: block = 64 columns x 4 split stripes (each stripe row a 256-B coalesced read).
// ---------------------------------------------------------------------------------------------
// Final value of one gradient column (+ its dot contributions). Lanes of wave 0 only.
__device__ __forceinline__ void ra_column(const RedAllArgs &a, const RedSeg &S, int cg, long long col, bool live,
                                          double colsum) {
  const int lane = threadIdx.x & 63;
  double d0 = 0.0, d1 = 0.0, d2 = 0.0;
  if (live) {
    const long long e = S.goff + col;
    float gv = S.splits > 0 ? float(colsum) : a.G[e];
    const float wv = (a.w && (a.dots || (a.l2 && a.lambda != 0.0))) ? a.w[e] : 0.0f;
    if (a.l2 && a.lambda != 0.0) gv = gv + float(a.lambda) * wv; // finalize_kernel's update
    if (a.dots) {
      d0 = double(gv) * double(gv);
      if (a.p) d1 = double(gv) * double(a.p[e]);
      d2 = double(wv) * double(wv);
    }
    if (S.splits > 0 || (a.l2 && a.lambda != 0.0)) a.G[e] = gv;
  }
  if (a.dots) {
    d0 = wave_sum(d0);
    d1 = wave_sum(d1);
    d2 = wave_sum(d2);
    if (lane == 0) {
      a.partials[cg * 3 + 0] = d0;
      a.partials[cg * 3 + 1] = d1;
      a.partials[cg * 3 + 2] = d2;
    }
  }
}

// Segments reduced in one pass (parts == 1) take RA_GPB column groups per block, four columns per lane:
// every load of the block (slab values, then the operands of ra_columns) is issued before its first use,
// and a quarter of the blocks of one group each (a 535,818-parameter gradient was 8,372 blocks, several
// rounds per CU).
template <int J>
__device__ __forceinline__ void ra_columns(const RedAllArgs &a, const RedSeg &S, int cg0, long long cgl0,
                                           const double (&colsum)[J]) {
  const int lane = threadIdx.x & 63;
  const bool need_w = a.w && (a.dots || (a.l2 && a.lambda != 0.0));
  const bool lam = a.l2 && a.lambda != 0.0;
  long long e[J];
  bool live[J];
  float gv[J], wv[J], pv[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const long long col = (cgl0 + j) * RA_COLS + lane;
    live[j] = col < S.count;
    e[j] = S.goff + (live[j] ? col : 0);
  }
#pragma unroll
  for (int j = 0; j < J; ++j) {
    gv[j] = S.splits > 0 ? float(colsum[j]) : a.G[e[j]];
    wv[j] = need_w ? a.w[e[j]] : 0.0f;
    pv[j] = (a.dots && a.p) ? a.p[e[j]] : 0.0f;
  }
#pragma unroll
  for (int j = 0; j < J; ++j) {
    if ((cgl0 + j) * RA_COLS >= S.count) break; // wave-uniform: past the segment's last group
    double d0 = 0.0, d1 = 0.0, d2 = 0.0;
    float g = gv[j];
    if (live[j]) {
      if (lam) g = g + float(a.lambda) * wv[j]; // finalize_kernel's update
      if (a.dots) {
        d0 = double(g) * double(g);
        if (a.p) d1 = double(g) * double(pv[j]);
        d2 = double(wv[j]) * double(wv[j]);
      }
      if (S.splits > 0 || lam) a.G[e[j]] = g;
    }
    if (a.dots) {
      d0 = wave_sum(d0);
      d1 = wave_sum(d1);
      d2 = wave_sum(d2);
      if (lane == 0) {
        const int cg = cg0 + j;
        a.partials[cg * 3 + 0] = d0;
        a.partials[cg * 3 + 1] = d1;
        a.partials[cg * 3 + 2] = d2;
      }
    }
  }
}

// One block of a single-pass segment: J column groups (J * 64 columns, one per lane per group).
template <int J>
__device__ __forceinline__ void ra_block(const RedAllArgs &a, const RedSeg &S, int local, double (*part)[RA_GPB * RA_COLS]) {
  const int t = threadIdx.x, lane = t & 63, stripe = t >> 6;
  const long long cgl0 = (long long)local * J;
  double acc[J];
  const float *src[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const long long col = (cgl0 + j) * RA_COLS + lane;
    acc[j] = 0.0;
    src[j] = S.slab + (col < S.count ? col : 0); // clamped; masked when used
  }
  if (S.splits > 0) {
    // the stripe's splits k = stripe, stripe + 4, ...: rounds of four (4 x J loads in flight), then the
    // last up-to-three from clamped splits, masked; summed in split order either way
    int k = stripe;
    for (; k + 12 < S.splits; k += 16) {
      float x[4][J];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < J; ++j) x[u][j] = src[j][(long long)(k + 4 * u) * S.stride];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < J; ++j) acc[j] += double(x[u][j]);
    }
    float x[3][J];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const long long kk = k + 4 * u < S.splits ? k + 4 * u : 0;
#pragma unroll
      for (int j = 0; j < J; ++j) x[u][j] = src[j][kk * S.stride];
    }
#pragma unroll
    for (int u = 0; u < 3; ++u)
      if (k + 4 * u < S.splits) // wave-uniform
#pragma unroll
        for (int j = 0; j < J; ++j) acc[j] += double(x[u][j]);
  }
#pragma unroll
  for (int j = 0; j < J; ++j) part[stripe][j * RA_COLS + lane] = acc[j];
  __syncthreads();
  if (stripe != 0) return;
  double colsum[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int q = j * RA_COLS + lane;
    colsum[j] = ((part[0][q] + part[1][q]) + part[2][q]) + part[3][q];
  }
  ra_columns<J>(a, S, S.cg0 + int(cgl0), cgl0, colsum);
}

// One wave (lane t < 64): the rank's SSE partials in a fixed order, stored as an fp32 (hi, lo) pair.
__device__ __forceinline__ void sse_pack_body(const double *sse_part, int nsse, float *hilo, int t) {
  double s = 0.0;
  for (int r = t; r < nsse; r += 64) s += sse_part[r];
  s = wave_sum(s);
  if (t == 0) {
    const float hi = float(s);
    hilo[0] = hi;
    hilo[1] = float(s - double(hi));
  }
}

__global__ __launch_bounds__(256) void reduce_all_kernel(const RedAllArgs a) {
  if (a.abort && *a.abort) return;
  __shared__ double part[4][RA_GPB * RA_COLS];
  const int t = threadIdx.x, lane = t & 63, stripe = t >> 6;
  const int b = blockIdx.x;
  if (b == a.nwg) { // the extra block of a data-parallel local reduction: the SSE words (sse_pack's launch)
    if (t < 64) sse_pack_body(a.sse_part, a.nsse, a.sse_hilo, t);
    return;
  }
  int si = 0;
  while (si + 1 < a.nseg && a.seg[si + 1].wg0 <= b) ++si;
  const RedSeg S = a.seg[si];
  const int local = b - S.wg0;
  if (S.parts == 1) { // wave-uniform
    if (S.gpb == RA_GPB) ra_block<RA_GPB>(a, S, local, part);
    else ra_block<1>(a, S, local, part);
    return;
  }
  const int cgl = local / S.parts, pi = local - cgl * S.parts;
  const int cg = S.cg0 + cgl;
  const long long col = (long long)cgl * RA_COLS + lane;
  const bool live = col < S.count;
  // this block's contiguous range of splits
  const int k0 = int((long long)S.splits * pi / S.parts), k1 = int((long long)S.splits * (pi + 1) / S.parts);
  double acc = 0.0;
  if (live && S.splits > 0) {
    const float *src = S.slab + col;
    int k = k0 + stripe;
    for (; k + 12 < k1; k += 16) { // four independent loads in flight, summed in split order
      const float x0 = src[(long long)k * S.stride], x1 = src[(long long)(k + 4) * S.stride];
      const float x2 = src[(long long)(k + 8) * S.stride], x3 = src[(long long)(k + 12) * S.stride];
      acc += double(x0);
      acc += double(x1);
      acc += double(x2);
      acc += double(x3);
    }
    for (; k < k1; k += 4) acc += double(src[(long long)k * S.stride]);
  }
  part[stripe][lane] = acc;
  __syncthreads();
  if (stripe != 0) return;
  const double colsum = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
  a.colpart[((long long)cg * RA_MAXPART + pi) * RA_COLS + lane] = colsum;
}

// One block: combine the split-range partials of the multi-range column groups, then (single rank)
// the eval_tail reduction. Everything it reads was written by earlier launches (stream order), so it
// needs no fence.
constexpr int RF_THREADS = 1024;
__global__ __launch_bounds__(RF_THREADS) void reduce_fin_kernel(const RedAllArgs a) {
  if (a.abort && *a.abort) return;
  KT(32);
  __shared__ double v[4];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  for (int b = wave; b < a.nfin; b += RF_THREADS / 64) {
    int si = 0;
    while (!(a.seg[si].fin0 >= 0 && b >= a.seg[si].fin0 &&
             b < a.seg[si].fin0 + int((a.seg[si].count + RA_COLS - 1) / RA_COLS)))
      ++si;
    const RedSeg S = a.seg[si];
    const int cgl = b - S.fin0, cg = S.cg0 + cgl;
    const long long col = (long long)cgl * RA_COLS + lane;
    double pv[RA_MAXPART];
#pragma unroll
    for (int q = 0; q < RA_MAXPART; ++q)
      pv[q] = q < S.parts ? a.colpart[((long long)cg * RA_MAXPART + q) * RA_COLS + lane] : 0.0;
    double colsum = 0.0;
#pragma unroll
    for (int q = 0; q < RA_MAXPART; ++q)
      if (q < S.parts) colsum += pv[q];
    ra_column(a, S, cg, col, col < S.count, colsum);
  }
  KT(33);
  if (!a.dots) return;
  __syncthreads(); // this block's partials are visible to the whole block
  KT(34);
  // every thread a fixed set of rows, then a fixed-order tree: deterministic, one round of loads
  __shared__ double ws[RF_THREADS / 64][4];
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int r = t; r < a.ncg; r += RF_THREADS) {
    acc[0] += a.partials[r * 3 + 0];
    acc[1] += a.partials[r * 3 + 1];
    acc[2] += a.partials[r * 3 + 2];
  }
  for (int r = t; r < a.nsse; r += RF_THREADS) acc[3] += a.sse_part[r];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const double w = wave_sum(acc[i]);
    if (lane == 0) ws[wave][i] = w;
  }
  __syncthreads();
  if (t < 4) {
    double x = 0.0;
    for (int w = 0; w < RF_THREADS / 64; ++w) x += ws[w][t];
    v[t] = x;
  }
  __syncthreads();
  if (t == 0) {
    double *sc = a.scal;
    sc[SC_TGG] = v[0];
    sc[SC_TGP] = v[1];
    sc[SC_WW] = v[2];
    sc[SC_SSE] = v[3];
    double loss = 0.5 * v[3] * a.inv_scale;
    if (a.lambda != 0.0) loss += 0.5 * a.lambda * v[2];
    sc[SC_LOSS] = loss;
  }
  KT(35);
}

// Forward-only loss of a line-search trial: the SSE partials summed exactly as reduce_fin_kernel sums
// them (same threads, same strided rows, same wave and cross-wave order), so the loss is bitwise the
// one the full evaluation of the same point reports; data parallel: from the all-reduced (hi, lo).
__global__ __launch_bounds__(RF_THREADS) void sse_loss_kernel(const double *sse_part, int nsse, const float *hilo,
                                                              double inv_scale, double *scal, const int *abort) {
  if (abort && *abort) return;
  __shared__ double ws[RF_THREADS / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  double acc = 0.0;
  if (!hilo)
    for (int r = t; r < nsse; r += RF_THREADS) acc += sse_part[r];
  const double w = wave_sum(acc);
  if (lane == 0) ws[wave] = w;
  __syncthreads();
  if (t == 0) {
    double x = 0.0;
    for (int i = 0; i < RF_THREADS / 64; ++i) x += ws[i];
    const double sse = hilo ? (double(hilo[0]) + double(hilo[1])) : x;
    scal[SC_SSE] = sse;
    scal[SC_LOSS] = 0.5 * sse * inv_scale;
  }
}
void sse_loss(hipStream_t s, const double *sse_part, int nsse, const float *hilo, double inv_scale, double *scal,
              const int *abort) {
  hipLaunchKernelGGL(sse_loss_kernel, dim3(1), dim3(RF_THREADS), 0, s, sse_part, nsse, hilo, inv_scale, scal, abort);
  LBF_KERNEL_CHECK();
}

void reduce_all(hipStream_t s, const RedAllArgs &a) {
  if (a.nwg <= 0 && !a.sse_hilo) return;
  hipLaunchKernelGGL(reduce_all_kernel, dim3(unsigned(a.nwg + (a.sse_hilo ? 1 : 0))), dim3(256), 0, s, a);
  LBF_KERNEL_CHECK();
  if (a.nfin > 0 || a.dots) {
    hipLaunchKernelGGL(reduce_fin_kernel, dim3(1), dim3(RF_THREADS), 0, s, a);
    LBF_KERNEL_CHECK();
  }
}

// ---------------------------------------------------------------------------------------------
// finalize: g += lambda*w (S-LBFGS L2 term, unified_optimization.hpp:375) ; partial (g.g, g.p, w.w)
// ---------------------------------------------------------------------------------------------
int dots_partials_wg(long long n) {
  long long w = cdiv(n, 256 * 8);
  return int(w < 1 ? 1 : (w > 512 ? 512 : w));
}

// g_in (nullable): read the gradient there and always write g (a data-parallel evaluation's all-reduced
// words buffer -> the live gradient, only when the speculative chain was not aborted)
__global__ __launch_bounds__(256) void finalize_kernel(long long n, float *g, const float *g_in, const float *w,
                                                       double lambda, const float *p, double *partials,
                                                       const int *abort) {
  if (abort && *abort) return;
  __shared__ double scratch[48];
  double acc[3] = {0.0, 0.0, 0.0};
  const long long stride = (long long)gridDim.x * blockDim.x;
  const float lf = float(lambda);
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    float gv = (g_in ? g_in : g)[e];
    const float wv = w ? w[e] : 0.0f;
    if (lambda != 0.0) gv = gv + lf * wv;
    if (lambda != 0.0 || g_in) g[e] = gv;
    acc[0] += double(gv) * double(gv);
    if (p) acc[1] += double(gv) * double(p[e]);
    acc[2] += double(wv) * double(wv);
  }
  block_sum<3>(acc, scratch);
  if (threadIdx.x == 0) {
    partials[blockIdx.x * 3 + 0] = acc[0];
    partials[blockIdx.x * 3 + 1] = acc[1];
    partials[blockIdx.x * 3 + 2] = acc[2];
  }
}

// G[r * ld + e] += lambda w[e] for r < rows, e < n: finalize_kernel's update (same fp32 expression) on
// each of a block of per-minibatch gradients (Mlp::batch_grads).
__global__ __launch_bounds__(256) void add_l2_rows_kernel(long long n, int rows, long long ld, float *G,
                                                          const float *w, double lambda) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const float lf = float(lambda), wv = w[e];
  float *g = G + e;
  // written as the fused multiply-add the contracted `gv + lf * wv` of finalize_kernel / reduce_all
  // compiles to (here the product is loop-invariant and would otherwise be hoisted and rounded once)
  for (int r = 0; r < rows; ++r) g[r * ld] = __builtin_fmaf(lf, wv, g[r * ld]);
}

void add_l2_rows(hipStream_t s, long long n, int rows, long long ld, float *G, const float *w, double lambda) {
  if (n <= 0 || rows <= 0 || lambda == 0.0) return;
  hipLaunchKernelGGL(add_l2_rows_kernel, dim3(unsigned(cdiv(n, 256))), dim3(256), 0, s, n, rows, ld, G, w, lambda);
  LBF_KERNEL_CHECK();
}

void finalize_grad_dots(hipStream_t s, long long n, float *g, const float *w, double lambda, const float *p,
                        double *partials, const int *abort, const float *g_in) {
  hipLaunchKernelGGL(finalize_kernel, dim3(dots_partials_wg(n)), dim3(256), 0, s, n, g, g_in, w, lambda, p, partials,
                     abort);
  LBF_KERNEL_CHECK();
}

__global__ __launch_bounds__(256) void dot_kernel(long long n, const float *x, const float *y, double *partials) {
  __shared__ double scratch[16];
  double acc[1] = {0.0};
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride)
    acc[0] += double(x[e]) * double(y[e]);
  block_sum<1>(acc, scratch);
  if (threadIdx.x == 0) partials[blockIdx.x] = acc[0];
}

void dot_partials(hipStream_t s, long long n, const float *x, const float *y, double *partials) {
  hipLaunchKernelGGL(dot_kernel, dim3(dots_partials_wg(n)), dim3(256), 0, s, n, x, y, partials);
  LBF_KERNEL_CHECK();
}

__global__ void eval_status_kernel(const double *sse_d, const float *hilo, double inv_scale, double lambda,
                                   double *scal) {
  const double sse = hilo ? (double(hilo[0]) + double(hilo[1])) : sse_d[0];
  scal[SC_SSE] = sse;
  double loss = 0.5 * sse * inv_scale;
  if (lambda != 0.0) loss += 0.5 * lambda * scal[SC_WW];
  scal[SC_LOSS] = loss;
}

void eval_status(hipStream_t s, const double *sse_d, const float *sse_hilo, double inv_scale, double lambda,
                 double *scal) {
  hipLaunchKernelGGL(eval_status_kernel, dim3(1), dim3(1), 0, s, sse_d, sse_hilo, inv_scale, lambda, scal);
  LBF_KERNEL_CHECK();
}

__global__ void pack_hilo_kernel(const double *x, float *hilo) {
  const float hi = float(x[0]);
  hilo[0] = hi;
  hilo[1] = float(x[0] - double(hi));
}
void pack_hilo(hipStream_t s, const double *x, float *hilo) {
  hipLaunchKernelGGL(pack_hilo_kernel, dim3(1), dim3(1), 0, s, x, hilo);
  LBF_KERNEL_CHECK();
}

// ---------------------------------------------------------------------------------------------
// BLAS-1 style helpers (vectorised; n tail handled per element)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void axpy_to_kernel(long long n, const float *x, float alpha, const float *p,
                                                      float *y) {
  const long long e = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (e + 3 < n) {
    const f32x4 a = *reinterpret_cast<const f32x4 *>(x + e);
    const f32x4 b = *reinterpret_cast<const f32x4 *>(p + e);
    *reinterpret_cast<f32x4 *>(y + e) = a + alpha * b;
  } else {
    for (long long j = e; j < n; ++j) y[j] = x[j] + alpha * p[j];
  }
}
// GD / SGD step (gd.cuh:77-85, sgd.cuh:115-124): v = m v - lr g ; x += v (m > 0), else x -= lr g. The
// reference's scal + two cuBLAS saxpys in one pass: v*m rounded, then the saxpys' fused multiply-adds.
// lr is read from the device (SGD's decayed rate lives there) when lr_dev is non-null.
__global__ __launch_bounds__(256) void momentum_step_kernel(long long n, float momentum, float lr, const float *lr_dev,
                                                            const float *g, float *v, float *x) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float r = lr_dev ? *lr_dev : lr;
  if (momentum > 0.0f) {
    const float vi = __fmaf_rn(-r, g[i], __fmul_rn(v[i], momentum));
    v[i] = vi;
    x[i] = __fadd_rn(x[i], vi);
  } else {
    x[i] = __fmaf_rn(-r, g[i], x[i]);
  }
}
void momentum_step(hipStream_t s, long long n, float momentum, float lr, const float *lr_dev, const float *g, float *v,
                   float *x) {
  if (n <= 0) return;
  hipLaunchKernelGGL(momentum_step_kernel, dim3(unsigned(cdiv(n, 256))), dim3(256), 0, s, n, momentum, lr, lr_dev, g,
                     v, x);
  LBF_KERNEL_CHECK();
}

// SGD's epoch loss (sgd.cuh:126): esum += float(batch loss) * float(batch rows), fp32 like the reference's
// host scalars; one thread, after each batch evaluation (no host round trip per batch).
__global__ void epoch_loss_acc_kernel(const double *scal, float rows, float *esum) {
  *esum = __fadd_rn(*esum, __fmul_rn(float(scal[SC_LOSS]), rows));
}
void epoch_loss_acc(hipStream_t s, const double *scal, long long rows, float *esum) {
  hipLaunchKernelGGL(epoch_loss_acc_kernel, dim3(1), dim3(1), 0, s, scal, float(rows), esum);
  LBF_KERNEL_CHECK();
}

void axpy_to(hipStream_t s, long long n, const float *x, float alpha, const float *p, float *y) {
  hipLaunchKernelGGL(axpy_to_kernel, dim3(unsigned(cdiv(cdiv(n, 4), 256))), dim3(256), 0, s, n, x, alpha, p, y);
  LBF_KERNEL_CHECK();
}
void axpy(hipStream_t s, long long n, float alpha, const float *x, float *y) { axpy_to(s, n, y, alpha, x, y); }

__global__ __launch_bounds__(256) void scal_kernel(long long n, float alpha, float *x) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) x[e] *= alpha;
}
void scal(hipStream_t s, long long n, float alpha, float *x) {
  hipLaunchKernelGGL(scal_kernel, dim3(unsigned(cdiv(n, 256))), dim3(256), 0, s, n, alpha, x);
  LBF_KERNEL_CHECK();
}

__global__ __launch_bounds__(256) void lincomb_kernel(long long n, const float *a, double c, const float *b,
                                                      float *out) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) out[e] = float(double(a[e]) + c * double(b[e]));
}
void lincomb(hipStream_t s, long long n, const float *a, double c, const float *b, float *out) {
  hipLaunchKernelGGL(lincomb_kernel, dim3(unsigned(cdiv(n, 256))), dim3(256), 0, s, n, a, c, b, out);
  LBF_KERNEL_CHECK();
}

// Minibatch rows gathered into a contiguous block (S-LBFGS: both evaluations of an inner step read the
// same rows; batch_g's column gather, unified_optimization.hpp:361-364). 16-B lanes when cols % 4 == 0,
// ld % 4 == 0 and both base pointers are 16-B aligned (the caller's X may be any float pointer).
__global__ __launch_bounds__(256) void gather_rows_kernel(const float *src, long long ld, const int *idx,
                                                          long long count, int cols, int vec, float *dst) {
  const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (vec) {
    const int c4 = cols >> 2;
    if (q >= count * c4) return;
    const long long r = q / c4, c = (q - r * c4) * 4;
    *reinterpret_cast<f32x4 *>(dst + r * cols + c) = *reinterpret_cast<const f32x4 *>(src + (long long)idx[r] * ld + c);
  } else {
    if (q >= count * cols) return;
    const long long r = q / cols, c = q - r * cols;
    dst[r * cols + c] = src[(long long)idx[r] * ld + c];
  }
}
void gather_rows(hipStream_t s, const float *src, long long ld, const int *idx, long long count, int cols,
                 float *dst) {
  if (count <= 0) return;
  const bool aligned = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15u) == 0;
  const int vec = (cols & 3) == 0 && (ld & 3) == 0 && aligned ? 1 : 0;
  const long long per = vec ? cols / 4 : cols;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(unsigned(cdiv(count * per, 256))), dim3(256), 0, s, src, ld, idx, count,
                     cols, vec, dst);
  LBF_KERNEL_CHECK();
}

// x[0 .. n) = 0 unless the speculative chain was aborted (a data-parallel rank's empty share)
__global__ __launch_bounds__(256) void zero_fill_kernel(long long n, float *x, const int *abort) {
  if (abort && *abort) return;
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) x[e] = 0.0f;
}
void zero_fill(hipStream_t s, long long n, float *x, const int *abort) {
  if (n <= 0) return;
  hipLaunchKernelGGL(zero_fill_kernel, dim3(unsigned(cdiv(n, 256))), dim3(256), 0, s, n, x, abort);
  LBF_KERNEL_CHECK();
}

// In-process rank group (comm.cpp LocalComm): dst = src[0] + src[1] + ... in rank order, fp32, so
// every rank of the group computes the same bits.
__global__ __launch_bounds__(256) void sum_ranks_kernel(RankSrcs r, long long count, float *dst) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  float acc = r.p[0][e];
  for (int i = 1; i < r.n; ++i) acc += r.p[i][e];
  dst[e] = acc;
}
void sum_ranks(hipStream_t s, const RankSrcs &r, long long count, float *dst) {
  LBF_REQUIRE(r.n >= 1 && r.n <= kMaxLocalRanks, "sum_ranks: 1..16 ranks");
  if (count <= 0) return;
  hipLaunchKernelGGL(sum_ranks_kernel, dim3(unsigned(cdiv(count, 256))), dim3(256), 0, s, r, count, dst);
  LBF_KERNEL_CHECK();
}

// Order-independent 32-bit fingerprints (a sum and an xor of mixed element bits) of x[0 .. n), stored in
// out[4 slot .. 4 slot + 3] as four exact 16-bit halves in floats, so that a sum all-reduce of a zeroed
// [4 nranks] buffer in which each rank filled its own slot hands every rank every rank's fingerprints.
// One workgroup: called once per S-LBFGS epoch (the replicated data-parallel check).
__global__ __launch_bounds__(1024) void fingerprint_kernel(long long n, const float *x, int slot, float *out) {
  const int t = threadIdx.x;
  unsigned hs = 0u, hx = 0u;
  for (long long e = t; e < n; e += 1024) {
    unsigned h = (__float_as_uint(x[e]) ^ (unsigned(e) * 0x9E3779B9u)) * 0x85EBCA6Bu;
    h ^= h >> 13;
    hs += h;
    hx ^= h * 0xC2B2AE35u;
  }
  __shared__ unsigned ss[1024], sx[1024];
  ss[t] = hs;
  sx[t] = hx;
  __syncthreads();
  for (int k = 512; k > 0; k >>= 1) {
    if (t < k) {
      ss[t] += ss[t + k];
      sx[t] ^= sx[t + k];
    }
    __syncthreads();
  }
  if (t < 4) {
    const unsigned v = t < 2 ? ss[0] : sx[0];
    out[4 * slot + t] = float((t & 1) ? (v >> 16) : (v & 0xffffu));
  }
}
void fingerprint(hipStream_t s, long long n, const float *x, int slot, float *out) {
  hipLaunchKernelGGL(fingerprint_kernel, dim3(1), dim3(1024), 0, s, n, x, slot, out);
  LBF_KERNEL_CHECK();
}

// y = (a - b) * scale in fp32: the pair sweep's y of a finite-difference HVP (gram_kernel forms the
// same product when it writes the ring slot)
__global__ __launch_bounds__(256) void diff_scale_kernel(long long n, const float *a, const float *b, float scale,
                                                         float *out) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) out[e] = (a[e] - b[e]) * scale;
}
void diff_scale(hipStream_t s, long long n, const float *a, const float *b, float scale, float *out) {
  hipLaunchKernelGGL(diff_scale_kernel, dim3(unsigned(cdiv(n, 256))), dim3(256), 0, s, n, a, b, scale, out);
  LBF_KERNEL_CHECK();
}

// S-LBFGS iterate averaging (s_lbfgs.hpp:236-243): u = (sum_i w_i) / cnt in logical order.
struct SlotList {
  int cnt;
  int slot[64];
};
__global__ __launch_bounds__(256) void average_kernel(long long n, const float *W, long long ld, SlotList sl,
                                                      float *u) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  double s = 0.0;
  for (int i = 0; i < sl.cnt; ++i) s += double(W[sl.slot[i] * ld + e]);
  u[e] = float(s / double(sl.cnt));
}
void average_slots(hipStream_t s, long long n, const float *W, long long ld, const int *h_slots, int cnt, float *u) {
  LBF_REQUIRE(cnt > 0 && cnt <= 64, "average_slots: 1..64 iterates supported (L+1 <= 64)");
  SlotList sl;
  sl.cnt = cnt;
  for (int i = 0; i < cnt; ++i) sl.slot[i] = h_slots[i];
  hipLaunchKernelGGL(average_kernel, dim3(unsigned(cdiv(n, 256))), dim3(256), 0, s, n, W, ld, sl, u);
  LBF_KERNEL_CHECK();
}

// ---------------------------------------------------------------------------------------------
// History: Gram sweep.
// Each workgroup owns a contiguous chunk of the n coordinates. Phase 1 forms the new vectors
// (s = sa - sb, y = (ya - yb)*yscale, g = ga - gb + gc) for the chunk into LDS, writes s/y into the
// ring slot (and g to g_out), and accumulates their 6 mutual dots. Phase 2 streams every live
// history vector once (one wave per vector, 8 waves) against the three LDS vectors.
// Partial columns per workgroup: live logical index i -> [S_i.s, Y_i.s, S_i.y, Y_i.y, S_i.g, Y_i.g]
// at 6*i..6*i+5 (i < m), then [s.s, s.y, y.y, g.s, g.y, g.g] at 6*m..6*m+5.
// ---------------------------------------------------------------------------------------------
// History loads: nontemporal (NT) when the ring is far larger than the 256 MB Infinity Cache, so the
// once-read stream does not evict what the evaluation keeps there (MI355X_MICROARCH.md nt-weights;
// profiles/micro/streams.hip: 5.2 -> 5.7 TB/s on the cfg-5 ring).
template <bool NT>
__device__ __forceinline__ f32x4 hist_load(const float *p) {
  const f32x4 *q = reinterpret_cast<const f32x4 *>(p);
  if constexpr (NT)
    return __builtin_nontemporal_load(q);
  else
    return *q;
}
static bool hist_nt(const HistView &h) { return double(2 * h.m) * double(h.ld) * 4.0 > 512.0 * 1024 * 1024; }

static constexpr int GRAM_THREADS = 512;
// Largest chunk per workgroup (3 x chunk x 4 B of LDS; 1024-8192-element chunks measured alike,
// profiles/r02/c4_chunk*.json).
static long long gram_max_chunk() { return 4096; }

int gram_ncols(int m) { return 6 * m + 6; }
template <int U, bool NT, int MODE = 0>
__global__ __launch_bounds__(GRAM_THREADS) void gram_kernel(const GramArgs a, long long chunk, double *partials, int tr,
                                                            int vec);
// Workgroups of the Gram sweep resident on the whole chip at the largest chunk (LDS-bound: 3 per CU), once.
static long long gram_slots() {
  static const long long slots = [] {
    int dev = 0, cus = 0, per = 0;
    LBF_HIP(hipGetDevice(&dev));
    LBF_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    LBF_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, gram_kernel<4, true>, GRAM_THREADS,
                                                         size_t(3 * gram_max_chunk()) * sizeof(float)));
    return (long long)std::max(1, cus) * std::max(1, per);
  }();
  return slots;
}
int gram_nwg(long long n) {
  long long w = cdiv(n, 1024);
  if (w > 2048) w = 2048;
  long long need = cdiv(n, gram_max_chunk());
  if (w < need) w = need;
  // More workgroups than the chip holds at once: a whole number of rounds, every round full (n = 10.49M:
  // 2561 chunks of 4096 were 3.33 rounds of 768 resident workgroups, the last a third full; now 3072 of
  // 3416), chunks still <= 4096.
  const long long slots = gram_slots();
  // (whole rounds of workgroups measured no faster than 4096-element chunks, 5.35-5.41 against 5.44-5.47 TB/s at
  // n = 10.49M, profiles/r06/h/; LBF_GRAM_ROUNDS=1 for the A/B)
  static const int whole_rounds = env_int("LBF_GRAM_ROUNDS", 0);
  if (whole_rounds && w > slots) w = cdiv(need, slots) * slots;
  return int(w < 1 ? 1 : w);
}
static long long gram_chunk(long long n, int nwg) { return cdiv(cdiv(n, nwg), 4) * 4; }


// The new vectors of one element: gram_kernel's arithmetic (s = sa - sb, y = (ya - yb) * yscale into the
// ring's write slot, g = ga - gb + gc into g_out), staged in LDS, self dots accumulated.
struct GramNew {
  float sv, yv, gv;
};
__device__ __forceinline__ GramNew gram_new(const GramArgs &a, float sa, float sb, float ya, float yb, float ga, float gb,
                                            float gc, float ysc) {
  GramNew r{0.f, 0.f, 0.f};
  if (a.has_pair) {
    r.sv = sa - sb;
    r.yv = (ya - yb) * ysc;
  }
  if (a.has_g) {
    r.gv = ga;
    if (a.gb) r.gv = r.gv - gb;
    if (a.gc) r.gv = r.gv + gc;
  }
  return r;
}

// tr: partials stored transposed, [ncols][gridDim.x] (each column contiguous for gram_fin's column sums);
// else [gridDim.x][ncols] (hist_step / fold_rows). vec: every operand and the ring 16-B aligned (host
// check), so the new vectors are formed from 16-B loads, all issued before the first use.
// MODE 0: the fused sweep (the new vectors formed into LDS and the ring, then the history). The split sweep
// (large n, gram_update): MODE 1 forms the new vectors, writes s, y into the ring slot (and g_out), and stores the
// self dots' partial row entries, with the same chunks, threads and block sum as MODE 0 (bitwise its self dots);
// MODE 2 then stages s, y, g of its chunk from memory into LDS and runs the history phase. The fused form's
// phase-1 stores, made between the history streams, cost the sweep far more than their bytes (5.2-5.7 TB/s
// against 5.8-6.0 split, profiles/micro/ring_ld.hip gram3p_*, profiles/r06/k2/).
template <int U, bool NT, int MODE>
__global__ __launch_bounds__(GRAM_THREADS) void gram_kernel(const GramArgs a, long long chunk, double *partials, int tr,
                                                            int vec) {
  if (a.h.abort && *a.h.abort) return;
  KT(16);
  extern __shared__ __attribute__((aligned(16))) float sh[];
  __shared__ double scratch[6 * 16];
  __shared__ int order[COEF_MAXK]; // the live slots in logical order, staged once: no global load per vector below
  float *ls = sh, *ly = sh + chunk, *lg = sh + 2 * chunk;
  const HistView &h = a.h;
  const int ncols = 6 * h.m + 6;
  const long long e0 = (long long)blockIdx.x * chunk;
  const long long e1 = min(h.n, e0 + chunk);
  const int len = int(e1 > e0 ? e1 - e0 : 0);
  const int w = hist_write_slot(h.ist, h.m, a.policy, a.reset);
  const int count = a.reset ? 0 : h.ist[IST_COUNT];
  if (blockIdx.x == 0 && threadIdx.x == 0) h.ist[IST_WSLOT] = w;
  for (int i = threadIdx.x; i < count; i += blockDim.x) order[i] = h.ist[IST_ORDER + i]; // visible after block_sum

  double self[6] = {0, 0, 0, 0, 0, 0};
  float *Sw = h.S + (long long)w * h.ld + e0;
  float *Yw = h.Y + (long long)w * h.ld + e0;
  const float ysc = float(a.yscale);
  auto put = [&](int i, const GramNew &r) {
    if (MODE == 0) {
      ls[i] = r.sv;
      ly[i] = r.yv;
      lg[i] = r.gv;
    }
    const double s = r.sv, y = r.yv, g = r.gv;
    self[0] += s * s;
    self[1] += s * y;
    self[2] += y * y;
    self[3] += g * s;
    self[4] += g * y;
    self[5] += g * g;
  };
  int i_scalar = 0;
  if (MODE == 2) { // staged: s, y from the ring slot MODE 1 wrote, g from g_out / ga (zeros where MODE 0 has them)
    const float *gsrc = (a.gb || a.gc) ? a.g_out : a.ga;
    if (vec) {
      const int nq = len >> 2;
      for (int q = threadIdx.x; q < nq; q += GRAM_THREADS) {
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        const f32x4 s4 = a.has_pair ? *reinterpret_cast<const f32x4 *>(Sw + 4 * q) : z;
        const f32x4 y4 = a.has_pair ? *reinterpret_cast<const f32x4 *>(Yw + 4 * q) : z;
        const f32x4 g4 = a.has_g ? *reinterpret_cast<const f32x4 *>(gsrc + e0 + 4 * q) : z;
        *reinterpret_cast<f32x4 *>(ls + 4 * q) = s4;
        *reinterpret_cast<f32x4 *>(ly + 4 * q) = y4;
        *reinterpret_cast<f32x4 *>(lg + 4 * q) = g4;
      }
      i_scalar = 4 * nq;
    }
    for (int i = i_scalar + int(threadIdx.x); i < len; i += blockDim.x) {
      ls[i] = a.has_pair ? Sw[i] : 0.f;
      ly[i] = a.has_pair ? Yw[i] : 0.f;
      lg[i] = a.has_g ? gsrc[e0 + i] : 0.f;
    }
    __syncthreads();
  } else if (vec) { // two quads per thread per round, all seven operand loads of both issued up front
    const int nq = len >> 2;
    const float *dflt = a.ga ? a.ga : a.sa; // null operands read this and are masked
    for (int q0 = threadIdx.x; q0 < nq; q0 += 2 * GRAM_THREADS) {
      f32x4 op[2][7];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int q = min(q0 + u * GRAM_THREADS, nq - 1);
        const long long e = e0 + 4LL * q;
        const float *src[7] = {a.sa, a.sb, a.ya, a.yb, a.ga, a.gb, a.gc};
#pragma unroll
        for (int j = 0; j < 7; ++j) op[u][j] = *reinterpret_cast<const f32x4 *>((src[j] ? src[j] : dflt) + e);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int q = q0 + u * GRAM_THREADS;
        if (q >= nq) break;
        f32x4 s4, y4, g4;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const GramNew r = gram_new(a, op[u][0][c], op[u][1][c], op[u][2][c], op[u][3][c], op[u][4][c], op[u][5][c],
                                     op[u][6][c], ysc);
          s4[c] = r.sv;
          y4[c] = r.yv;
          g4[c] = r.gv;
          put(4 * q + c, r);
        }
        if (a.has_pair) {
          *reinterpret_cast<f32x4 *>(Sw + 4 * q) = s4;
          *reinterpret_cast<f32x4 *>(Yw + 4 * q) = y4;
        }
        if (a.has_g && a.g_out) *reinterpret_cast<f32x4 *>(a.g_out + e0 + 4 * q) = g4;
      }
    }
    i_scalar = 4 * nq;
  }
  if (MODE != 2)
    for (int i = i_scalar + int(threadIdx.x); i < len; i += blockDim.x) {
      const long long e = e0 + i;
      const GramNew r = gram_new(a, a.has_pair ? a.sa[e] : 0.f, a.has_pair ? a.sb[e] : 0.f, a.has_pair ? a.ya[e] : 0.f,
                                 a.has_pair ? a.yb[e] : 0.f, a.has_g ? a.ga[e] : 0.f, a.gb ? a.gb[e] : 0.f,
                                 a.gc ? a.gc[e] : 0.f, ysc);
      if (a.has_pair) {
        Sw[i] = r.sv;
        Yw[i] = r.yv;
      }
      if (a.has_g && a.g_out) a.g_out[e] = r.gv;
      put(i, r);
    }
  KT(17);
  const long long rs = tr ? (long long)gridDim.x : 1LL; // column stride of the partial table
  double *out = partials + (tr ? (long long)blockIdx.x : (long long)blockIdx.x * ncols);
  if (MODE != 2) {
    block_sum<6>(self, scratch); // includes __syncthreads: LDS vectors complete after this
    KT(18);
    if (threadIdx.x == 0)
      for (int j = 0; j < 6; ++j) out[(6 * h.m + j) * rs] = self[j];
    if (MODE == 1) return;
  }

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int v = wave; v < 2 * count; v += nw) {
    const int li = v < count ? v : v - count;
    const int slot = order[li];
    if (a.has_pair && slot == w) { // overwritten in this sweep (CUDA full ring): dots from the self block
      if (lane == 0) {
        out[(6 * li + (v < count ? 0 : 1)) * rs] = 0.0;
        out[(6 * li + (v < count ? 2 : 3)) * rs] = 0.0;
        out[(6 * li + (v < count ? 4 : 5)) * rs] = 0.0;
      }
      continue;
    }
    const float *V = (v < count ? h.S : h.Y) + (long long)slot * h.ld + e0;
    double ds = 0.0, dy = 0.0, dg = 0.0;
    const int full = len & ~3; // elements in whole 16-B quads
    for (int i0 = lane * 4; i0 < full; i0 += 256 * U) { // U independent 16-B loads in flight per lane
      f32x4 xs[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int iu = i0 + 256 * u;
        xs[u] = hist_load<NT>(V + (iu < full ? iu : 0)); // clamped, masked below: no per-load branch
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int iu = i0 + 256 * u;
        if (iu < full) {
          const f32x4 s4 = *reinterpret_cast<const f32x4 *>(ls + iu);
          const f32x4 y4 = *reinterpret_cast<const f32x4 *>(ly + iu);
          const f32x4 g4 = *reinterpret_cast<const f32x4 *>(lg + iu);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const double xv = xs[u][j];
            ds += xv * double(s4[j]);
            dy += xv * double(y4[j]);
            dg += xv * double(g4[j]);
          }
        }
      }
    }
    if (full < len && lane == ((full >> 2) & 63)) { // the partial quad, on the lane whose stride reaches it
      for (int j = full; j < len; ++j) {
        const double xv = V[j];
        ds += xv * double(ls[j]);
        dy += xv * double(ly[j]);
        dg += xv * double(lg[j]);
      }
    }
    ds = wave_sum(ds);
    dy = wave_sum(dy);
    dg = wave_sum(dg);
    if (lane == 0) {
      const int c = v < count ? 0 : 1;
      out[(6 * li + c + 0) * rs] = ds;
      out[(6 * li + c + 2) * rs] = dy;
      out[(6 * li + c + 4) * rs] = dg;
    }
  }
  KT(19);
}

void gram_update(hipStream_t s, const GramArgs &a, double *partials, int transposed) {
  const int nwg = gram_nwg(a.h.n);
  const long long chunk = gram_chunk(a.h.n, nwg);
  const size_t shmem = size_t(3 * chunk) * sizeof(float);
  // 16-B loads in flight per lane while streaming a history vector (8 measured the same as 4,
  // profiles/r03/two_loop_gramU8.jsonl)
  if (shmem > 64 * 1024) { // once per process, thread-safe
    static const bool attr_set = [] {
      for (const void *f : {reinterpret_cast<const void *>(gram_kernel<4, false>),
                            reinterpret_cast<const void *>(gram_kernel<4, true>),
                            reinterpret_cast<const void *>(gram_kernel<4, false, 2>),
                            reinterpret_cast<const void *>(gram_kernel<4, true, 2>)})
        LBF_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024));
      return true;
    }();
    (void)attr_set;
  }
  const bool nt = hist_nt(a.h);
  auto al16 = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }; // null passes
  const int vec = (a.ga || a.sa) && chunk % 4 == 0 && a.h.ld % 4 == 0 && al16(a.h.S) && al16(a.h.Y) &&
                  al16(a.sa) && al16(a.sb) && al16(a.ya) && al16(a.yb) && al16(a.ga) && al16(a.gb) && al16(a.gc) &&
                  al16(a.g_out);
  const int tr = transposed ? 1 : 0;
  // the split sweep (MODE 1 then 2) for the large-n history, where g is readable afterwards (ga, or g_out when formed)
  static const int split_on = env_int("LBF_GRAM_SPLIT", 1); // A/B: 0 keeps the fused sweep
  // (long histories only: at m = 10 the extra launch and the three staged reads cost what the split saves, two-loop
  // 56.9-57.5 % split against 57.1-58.1 % fused; m = 50 68.9-69.6 % against 67.2-67.3 %, profiles/r06/m/)
  if (split_on && vec && a.h.n >= (1LL << 21) && a.h.m >= 20 && !(a.has_g && (a.gb || a.gc) && !a.g_out)) {
    const dim3 g1{unsigned(nwg), 1, 1}, b1{unsigned(GRAM_THREADS), 1, 1};
    if (nt) {
      hipLaunchKernelGGL((gram_kernel<4, true, 1>), g1, b1, 0, s, a, chunk, partials, tr, vec);
      hipLaunchKernelGGL((gram_kernel<4, true, 2>), g1, b1, shmem, s, a, chunk, partials, tr, vec);
    } else {
      hipLaunchKernelGGL((gram_kernel<4, false, 1>), g1, b1, 0, s, a, chunk, partials, tr, vec);
      hipLaunchKernelGGL((gram_kernel<4, false, 2>), g1, b1, shmem, s, a, chunk, partials, tr, vec);
    }
    LBF_KERNEL_CHECK();
    return;
  }
  if (nt)
    hipLaunchKernelGGL((gram_kernel<4, true>), dim3(nwg), dim3(GRAM_THREADS), shmem, s, a, chunk, partials, tr, vec);
  else
    hipLaunchKernelGGL((gram_kernel<4, false>), dim3(nwg), dim3(GRAM_THREADS), shmem, s, a, chunk, partials, tr, vec);
  LBF_KERNEL_CHECK();
}

// ---------------------------------------------------------------------------------------------
// History step (one workgroup): (A) reduce the Gram sweep's per-workgroup partials, then the push and
// the two-loop recurrences of hist_core.hpp.
// ---------------------------------------------------------------------------------------------
static constexpr int HIST_STAGE_DOUBLES = 4096;   // up to 32 KB of partial rows staged per round
static constexpr int HIST_STATIC_LDS = 16 * 1024; // bound on the kernel's static LDS
static constexpr int HIST_PRE_UNROLL = 11;        // fused path: (m+1)^2 <= 256 * 11, i.e. m <= 52

__global__ __launch_bounds__(256) void hist_step_kernel(const CoefArgs a) {
  if (a.h.abort && *a.h.abort) return;
  KT(0);
  extern __shared__ double sy[]; // [k][k] live s_i . y_j after the push (logical order), then staging
  __shared__ HistSmem sm;
  const HistView &h = a.h;
  const int t = threadIdx.x;
  HistStep st;
  st.h = a.h;
  st.has_pair = a.has_pair;
  st.has_g = a.has_g;
  st.reset = a.reset;
  st.policy = a.policy;
  st.want_dir = a.want_dir;
  st.iter = a.iter;
  st.dsign = a.dsign;
  // fused: SY, YY and rho go to LDS (after the SY block and the staging area) with the prologue's
  // loads, one round trip for all of them; the recurrences then read LDS only
  constexpr int PU = HIST_PRE_UNROLL;
  const int S_ = h.slots, SS = S_ * S_;
  double *pre = sy + a.sy_cap + a.stage;
  double psy[PU], pyy[PU], prho = 0.0;
  if (a.fused) {
#pragma unroll
    for (int u = 0; u < PU; ++u) { // clamped, unconditional: no branch and wait per load
      const int i = min(t + 256 * u, SS - 1);
      psy[u] = h.SY[i];
      pyy[u] = h.YY[i];
    }
    prho = h.rho[min(t, S_ - 1)];
  }
  // Step A's partial rows in the same round trip when they fit one staging round (the folded table, History::
  // update): every column, the live ones picked after the prologue
  constexpr int AU = HIST_STAGE_DOUBLES / 256;
  const int ncols = 6 * h.m + 6, tot_all = a.nwg * ncols;
  const bool one_round = tot_all <= a.stage && tot_all <= 256 * AU;
  double pa[AU];
  if (one_round) {
#pragma unroll
    for (int u = 0; u < AU; ++u) pa[u] = a.partials[min(t + 256 * u, tot_all - 1)];
  }
  hist_prologue(st, sm, h.ist[IST_WSLOT]);
  if (a.fused) {
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const int i = t + 256 * u;
      if (i < SS) {
        pre[i] = psy[u];
        pre[SS + i] = pyy[u];
      }
    }
    if (t < S_) pre[2 * SS + t] = prho;
  }
  KT(1);
  const int count0 = sm.count0;
  // ---- A: reduce the columns in use. Tiles of partial rows are staged into LDS with every load in
  // flight at once (one global round trip per tile), then thread q sums column q in row order. ----
  const int nneed = 6 * count0 + 6;
  double *stage = sy + a.sy_cap; // dynamic LDS after the SY block(s)
  const int rt = max(1, min(a.nwg, a.stage / nneed));
  double colacc[(6 * COEF_MAXK + 6 + 255) / 256];
#pragma unroll
  for (int i = 0; i < (6 * COEF_MAXK + 6 + 255) / 256; ++i) colacc[i] = 0.0;
  if (one_round) { // the same sums in the same row order as the rounds below
#pragma unroll
    for (int u = 0; u < AU; ++u)
      if (t + 256 * u < tot_all) stage[t + 256 * u] = pa[u];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < (6 * COEF_MAXK + 6 + 255) / 256; ++i) {
      const int q = t + 256 * i;
      if (q < nneed) {
        const int col = q < 6 * count0 ? q : 6 * h.m + (q - 6 * count0);
        for (int r = 0; r < a.nwg; ++r) colacc[i] += stage[r * ncols + col];
      }
    }
    __syncthreads();
  }
  for (int r0 = 0; !one_round && r0 < a.nwg; r0 += rt) {
    const int rows = min(rt, a.nwg - r0);
    const int tot = rows * nneed;
    for (int e0 = t; e0 < tot; e0 += 256 * 8) { // 8 independent loads in flight per thread
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) { // unconditional (clamped) loads: no branch and wait per load
        const int e = min(e0 + 256 * u, tot - 1);
        const int r = e / nneed, q = e - r * nneed;
        const int col = q < 6 * count0 ? q : 6 * h.m + (q - 6 * count0);
        v[u] = a.partials[(long long)(r0 + r) * ncols + col];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (e0 + 256 * u < tot) stage[e0 + 256 * u] = v[u];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < (6 * COEF_MAXK + 6 + 255) / 256; ++i) {
      const int q = t + 256 * i;
      if (q < nneed)
        for (int r = 0; r < rows; ++r) colacc[i] += stage[r * nneed + q];
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < (6 * COEF_MAXK + 6 + 255) / 256; ++i) {
    const int q = t + 256 * i;
    if (q < nneed) sm.dots[q < 6 * count0 ? q : 6 * h.m + (q - 6 * count0)] = colacc[i];
  }
  __syncthreads();
  KT(2);
  if (a.fused) {
    st.SY = pre;
    st.YY = pre + SS;
    st.rho = pre + 2 * SS;
    hist_core<true>(st, sm, sy, a.sy_cap, stage, a.stage);
  } else {
    hist_core<false>(st, sm, sy, a.sy_cap, stage, a.stage);
  }
}

// Partial rows of the Gram table that one staging round of the history step holds (History::update
// folds taller tables to this many rows first, so step A is one round trip).
int hist_stage_rows(int m) {
  const long long total = (160 * 1024 - HIST_STATIC_LDS) / 8, m2 = (long long)m * m;
  const long long need_stage = 6LL * m + 6, S = m + 1, pre = 2 * S * S + S;
  const bool fused = S * S <= 256LL * HIST_PRE_UNROLL && 2 * m2 + HIST_STAGE_DOUBLES + pre <= total;
  const long long avail = total - (fused ? pre : 0);
  const long long big = (long long)m * (m + 1) + ((long long)m * (m + 1)) / 2;
  long long sy_cap;
  if (2 * m2 + HIST_STAGE_DOUBLES <= avail || big + 4 * need_stage > avail)
    sy_cap = std::min(2 * m2, avail - need_stage);
  else
    sy_cap = big;
  const long long stage = std::min<long long>(HIST_STAGE_DOUBLES, avail - sy_cap);
  return int(std::max(1LL, stage / need_stage));
}

void hist_coef(hipStream_t s, const CoefArgs &a) {
  LBF_REQUIRE(a.h.m <= COEF_MAXK, "history size m must be <= 128");
  static const bool attr_set = [] { // once per process, thread-safe
    LBF_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(hist_step_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - HIST_STATIC_LDS));
    return true;
  }();
  (void)attr_set;
  CoefArgs c = a;
  const long long total = (160 * 1024 - HIST_STATIC_LDS) / 8, m2 = (long long)a.h.m * a.h.m;
  const long long need_stage = 6LL * a.h.m + 6;
  const long long S = a.h.slots, pre = 2 * S * S + S;
  // fused history step (LDS-prefetched sources, stores off wave 0) when the direction is wanted and
  // SY (with its transpose), a full staging area and the prefetch all fit
  c.fused = (a.want_dir == 1 && S * S <= 256LL * HIST_PRE_UNROLL &&
             2 * m2 + HIST_STAGE_DOUBLES + pre <= total) ? 1 : 0;
  const long long avail = total - (c.fused ? pre : 0);
  // SY and its transpose when they fit beside a full staging area; else (m = 100) hist_core's compact
  // layout (SY with stride m + 1, YY's lower triangle) so that step A keeps a staging area of many rows
  const long long big = (long long)a.h.m * (a.h.m + 1) + ((long long)a.h.m * (a.h.m + 1)) / 2;
  if (2 * m2 + HIST_STAGE_DOUBLES <= avail || big + 4 * need_stage > avail)
    c.sy_cap = int(std::min(2 * m2, avail - need_stage)); // SY, and its transpose when it fits
  else
    c.sy_cap = int(big);
  LBF_REQUIRE(c.sy_cap >= m2, "hist_step: LDS too small for the SY block");
  c.stage = int(std::min<long long>(HIST_STAGE_DOUBLES, avail - c.sy_cap));
  const size_t shmem = (size_t(c.sy_cap) + size_t(c.stage) + (c.fused ? size_t(pre) : 0)) * sizeof(double);
  hipLaunchKernelGGL(hist_step_kernel, dim3(1), dim3(256), shmem, s, c);
  LBF_KERNEL_CHECK();
}
// ---------------------------------------------------------------------------------------------
// History: linear-combination sweep  dir = sum_i cs_i S_i + cy_i Y_i + cg g  (fp64 per element),
// fused with the trial point x_out = x_in + alpha*dir (and an optional second copy).
// ---------------------------------------------------------------------------------------------
template <int U, bool NT>
__global__ __launch_bounds__(256) void combine_kernel(const CombineArgs a) {
  if (a.h.abort && *a.h.abort) return;
  __shared__ double cs[COEF_MAXK], cy[COEF_MAXK];
  __shared__ int L[COEF_MAXK];
  const HistView &h = a.h;
  const int S_ = h.slots;
  const int k = h.ist[IST_COUNT];
  for (int i = threadIdx.x; i < k; i += blockDim.x) {
    cs[i] = h.coef[i];
    cy[i] = h.coef[S_ + i];
    L[i] = h.ist[IST_ORDER + i];
  }
  __syncthreads();
  const double cg = h.coef[2 * S_];
  const double alpha = a.alpha_from_state ? h.scal[SC_ALPHA0] : a.alpha;
  // grid-stride over 16-B quads: the grid is the chip's resident workgroups, so every one takes the same
  // number of quads (within one) and there is no partly filled last round
  const long long stride = (long long)gridDim.x * blockDim.x * 4;
  for (long long e = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4; e < h.n; e += stride) {
  if (e + 3 < h.n) {
    const f32x4 g4 = *reinterpret_cast<const f32x4 *>(a.g + e);
    const f32x4 x4 = *reinterpret_cast<const f32x4 *>((a.x_out ? a.x_in : a.g) + e); // unconditional: no early wait
    double acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = cg * double(g4[j]);
    int i = 0;
    for (; i + U <= k; i += U) { // 2U independent 16-B loads in flight per lane
      f32x4 s4[U], y4[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        s4[u] = hist_load<NT>(h.S + (long long)L[i + u] * h.ld + e);
        y4[u] = hist_load<NT>(h.Y + (long long)L[i + u] * h.ld + e);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] += cs[i + u] * double(s4[u][j]) + cy[i + u] * double(y4[u][j]);
    }
    for (; i < k; ++i) {
      const f32x4 s4 = *reinterpret_cast<const f32x4 *>(h.S + (long long)L[i] * h.ld + e);
      const f32x4 y4 = *reinterpret_cast<const f32x4 *>(h.Y + (long long)L[i] * h.ld + e);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] += cs[i] * double(s4[j]) + cy[i] * double(y4[j]);
    }
    f32x4 d4;
#pragma unroll
    for (int j = 0; j < 4; ++j) d4[j] = float(acc[j]);
    if (a.dir) *reinterpret_cast<f32x4 *>(a.dir + e) = d4;
    if (a.x_out) {
      const f32x4 o4 = x4 + float(alpha) * d4;
      *reinterpret_cast<f32x4 *>(a.x_out + e) = o4;
      if (a.x_out2) *reinterpret_cast<f32x4 *>(a.x_out2 + e) = o4;
    }
  } else {
    for (long long q = e; q < h.n; ++q) {
      double acc = cg * double(a.g[q]);
      for (int i = 0; i < k; ++i)
        acc += cs[i] * double(h.S[(long long)L[i] * h.ld + q]) + cy[i] * double(h.Y[(long long)L[i] * h.ld + q]);
      const float d = float(acc);
      if (a.dir) a.dir[q] = d;
      if (a.x_out) {
        const float o = a.x_in[q] + float(alpha) * d;
        a.x_out[q] = o;
        if (a.x_out2) a.x_out2[q] = o;
      }
    }
  }
  }
}

// Large-n combine with the Gram sweep's access pattern (round 6). combine_kernel above reads, per wave-instruction,
// 1 KB of one vector and per lane one quad of every live vector, the grid striding over the elements: the chip
// then touches every vector at the same few offsets at once, a pattern that streams at 5.45 TB/s against 6.7 TB/s
// for the Gram sweep's (each wave 4-16 KB contiguous of one vector; profiles/micro/ring_ld.hip, profiles/r06/d/).
// Here a workgroup owns 4096-element chunks (grid-stride over the resident grid): wave w the 1024 elements
// c0 + 1024 w .., lane l the quads 256 u + 4 l (u < 4), so each vector is read as 4 KB contiguous per wave and
// 16 KB per workgroup, V vectors' quads (2 V x 4 loads) in flight per lane. Per element the same fp64 sum in the
// same order as combine_kernel (cg g, then cs_i S_i + cy_i Y_i for i = 0 .. k - 1).
template <int V, bool NT, int Q = 4>
__global__ __launch_bounds__(256) void combine_chunk_kernel(const CombineArgs a) {
  if (a.h.abort && *a.h.abort) return;
  __shared__ double cs[COEF_MAXK], cy[COEF_MAXK];
  __shared__ int L[COEF_MAXK];
  const HistView &h = a.h;
  const int S_ = h.slots;
  const int k = h.ist[IST_COUNT];
  for (int i = threadIdx.x; i < k; i += blockDim.x) {
    cs[i] = h.coef[i];
    cy[i] = h.coef[S_ + i];
    L[i] = h.ist[IST_ORDER + i];
  }
  __syncthreads();
  const double cg = h.coef[2 * S_];
  const double alpha = a.alpha_from_state ? h.scal[SC_ALPHA0] : a.alpha;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float *xsrc = a.x_out ? a.x_in : a.g;
  constexpr int CH = 1024 * Q; // elements per chunk: wave w the 256 Q contiguous elements c0 + 256 Q w ..
  for (long long c0 = (long long)blockIdx.x * CH; c0 < h.n; c0 += (long long)gridDim.x * CH) {
    long long e[Q], ec[Q];
    bool full[Q];
#pragma unroll
    for (int u = 0; u < Q; ++u) {
      e[u] = c0 + wave * 256 * Q + u * 256 + 4 * lane;
      full[u] = e[u] + 3 < h.n;
      ec[u] = full[u] ? e[u] : 0; // clamped: loads unconditional, results masked
    }
    double acc[Q][4];
#pragma unroll
    for (int u = 0; u < Q; ++u) {
      const f32x4 g4 = *reinterpret_cast<const f32x4 *>(a.g + ec[u]);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[u][j] = cg * double(g4[j]);
    }
    int i = 0;
    for (; i + V <= k; i += V) {
      f32x4 s4[V][Q], y4[V][Q];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const long long sb = (long long)L[i + v] * h.ld;
#pragma unroll
        for (int u = 0; u < Q; ++u) {
          s4[v][u] = hist_load<NT>(h.S + sb + ec[u]);
          y4[v][u] = hist_load<NT>(h.Y + sb + ec[u]);
        }
      }
#pragma unroll
      for (int v = 0; v < V; ++v)
#pragma unroll
        for (int u = 0; u < Q; ++u)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[u][j] += cs[i + v] * double(s4[v][u][j]) + cy[i + v] * double(y4[v][u][j]);
    }
    for (; i < k; ++i) {
      const long long sb = (long long)L[i] * h.ld;
#pragma unroll
      for (int u = 0; u < Q; ++u) {
        const f32x4 s4 = hist_load<NT>(h.S + sb + ec[u]);
        const f32x4 y4 = hist_load<NT>(h.Y + sb + ec[u]);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[u][j] += cs[i] * double(s4[j]) + cy[i] * double(y4[j]);
      }
    }
#pragma unroll
    for (int u = 0; u < Q; ++u) {
      if (full[u]) {
        f32x4 d4;
#pragma unroll
        for (int j = 0; j < 4; ++j) d4[j] = float(acc[u][j]);
        if (a.dir) *reinterpret_cast<f32x4 *>(a.dir + e[u]) = d4;
        if (a.x_out) {
          const f32x4 x4 = *reinterpret_cast<const f32x4 *>(xsrc + e[u]);
          const f32x4 o4 = x4 + float(alpha) * d4;
          *reinterpret_cast<f32x4 *>(a.x_out + e[u]) = o4;
          if (a.x_out2) *reinterpret_cast<f32x4 *>(a.x_out2 + e[u]) = o4;
        }
      } else {
        for (long long q = e[u]; q < h.n && q < e[u] + 4; ++q) { // the tail quad, element-wise (no read past n)
          double ac = cg * double(a.g[q]);
          for (int ii = 0; ii < k; ++ii)
            ac += cs[ii] * double(h.S[(long long)L[ii] * h.ld + q]) + cy[ii] * double(h.Y[(long long)L[ii] * h.ld + q]);
          const float d = float(ac);
          if (a.dir) a.dir[q] = d;
          if (a.x_out) {
            const float o = a.x_in[q] + float(alpha) * d;
            a.x_out[q] = o;
            if (a.x_out2) a.x_out2[q] = o;
          }
        }
      }
    }
  }
}

// Small-n form (the latency-bound regime: n up to a few million, k <= 32): one element per lane so
// the grid covers every CU, the ring header and coefficients read lane-distributed (no LDS, no
// barrier) and broadcast with v_readlane, and every history load of the lane issued at once: one
// round trip for the header, one for the data.
template <int KMAX>
__global__ __launch_bounds__(256) void combine_small_kernel(const CombineArgs a) {
  // the speculative chain's abort flag: requested with the header, g and x (one round trip for all) and
  // tested before the history loads, so an aborted launch exits after that round trip
  const int abf = abort_flag(a.h.abort);
  const HistView &h = a.h;
  const int S_ = h.slots, lane = threadIdx.x & 63;
  const long long e0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = e0 < h.n;
  const long long e = in ? e0 : h.n - 1; // loads are unconditional (clamped), results masked
  // independent of the header: in flight with it
  const float gv = a.g[e];
  const float xv = (a.x_out ? a.x_in : a.g)[e];
  const int lk = lane < h.m ? lane : 0; // header entries read without waiting for the count
  const int k = __builtin_amdgcn_readfirstlane(h.ist[IST_COUNT]);
  const int Lr = h.ist[IST_ORDER + lk];
  const double csr = h.coef[lk], cyr = h.coef[S_ + lk];
  const double cg = h.coef[2 * S_];
  const double alpha = a.alpha_from_state ? h.scal[SC_ALPHA0] : a.alpha;
  if (aborted(abf)) return; // uniform for the launch
  float sv[KMAX], yv[KMAX];
  if (k > 0) {
#pragma unroll
    for (int i = 0; i < KMAX; ++i) { // every load issued before the first use
      const long long off = (long long)__builtin_amdgcn_readlane(Lr, i < k ? i : k - 1) * h.ld + e;
      sv[i] = h.S[off];
      yv[i] = h.Y[off];
    }
  }
  double acc = cg * double(gv);
#pragma unroll
  for (int i = 0; i < KMAX; ++i)
    if (i < k) acc += lane_f64(csr, i) * double(sv[i]) + lane_f64(cyr, i) * double(yv[i]);
  if (!in) return;
  const float d = float(acc);
  if (a.dir) a.dir[e] = d;
  if (a.x_out) {
    const float o = xv + float(alpha) * d;
    a.x_out[e] = o;
    if (a.x_out2) a.x_out2[e] = o;
  }
}

void hist_combine(hipStream_t s, const CombineArgs &a) {
  LBF_REQUIRE(a.h.ld % 4 == 0, "history slot stride must be a multiple of 4");
  if (a.h.n <= (1LL << 21) && a.h.m <= 32) {
    const dim3 g1(unsigned(cdiv(a.h.n, 256)));
    if (a.h.m <= 16)
      hipLaunchKernelGGL(combine_small_kernel<16>, g1, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL(combine_small_kernel<32>, g1, dim3(256), 0, s, a);
    LBF_KERNEL_CHECK();
    return;
  }
  static const int chunked = env_int("LBF_COMBINE_CHUNK", 1); // A/B: 0 keeps combine_kernel
  if (chunked) {
    // 2 vectors x 4 quads in flight per lane: measured against 1 x 4, 2 x 2 and 4 x 2 (m = 50: 69.9-70.0 % against
    // 69.5-69.9, 67.3-67.6, 66.7-66.8 %; profiles/r06/o/)
    static const long long res_c = [] { // workgroups of combine_chunk_kernel the chip holds at once, once
      int dev = 0, cus = 0, p1 = 0, p2 = 0;
      LBF_HIP(hipGetDevice(&dev));
      LBF_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
      LBF_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&p1, combine_chunk_kernel<2, true, 4>, 256, 0));
      LBF_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&p2, combine_chunk_kernel<2, false, 4>, 256, 0));
      return (long long)std::max(1, cus) * std::max(1, std::min(p1, p2));
    }();
    const dim3 grid(unsigned(std::min(cdiv(a.h.n, 4096LL), res_c)));
    if (hist_nt(a.h))
      hipLaunchKernelGGL((combine_chunk_kernel<2, true, 4>), grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((combine_chunk_kernel<2, false, 4>), grid, dim3(256), 0, s, a);
    LBF_KERNEL_CHECK();
    return;
  }
  static const long long resident = [] { // workgroups of combine_kernel the chip holds at once, once
    int dev = 0, cus = 0, p8 = 0, p4 = 0;
    LBF_HIP(hipGetDevice(&dev));
    LBF_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    LBF_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&p8, combine_kernel<8, true>, 256, 0));
    LBF_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&p4, combine_kernel<4, false>, 256, 0));
    return (long long)std::max(1, cus) * std::max(1, std::min(p8, p4));
  }();
  const dim3 grid(unsigned(std::min(cdiv(cdiv(a.h.n, 4), 256), resident)));
  if (hist_nt(a.h))
    hipLaunchKernelGGL((combine_kernel<8, true>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((combine_kernel<4, false>), grid, dim3(256), 0, s, a);
  LBF_KERNEL_CHECK();
}

__global__ void hist_reset_kernel(HistView h) {
  h.ist[IST_COUNT] = 0;
  h.ist[IST_FREE] = 0;
  h.ist[IST_WSLOT] = 0;
  h.scal[SC_COUNT] = 0.0;
}
void hist_reset(hipStream_t s, const HistView &h) {
  hipLaunchKernelGGL(hist_reset_kernel, dim3(1), dim3(1), 0, s, h);
  LBF_KERNEL_CHECK();
}

// ---------------------------------------------------------------------------------------------
// Evaluation tail (one workgroup): fixed-order reductions of the finalize dots (g.g, g.p, w.w) and,
// on a single rank, of the SSE partials; then the loss (0.5*sse*inv_scale + 0.5*lambda*w.w).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void eval_tail_kernel(const double *dots_part, int nd, const double *sse_part,
                                                        int nsse, const float *hilo, double inv_scale,
                                                        double lambda, double *scal, const int *abort) {
  if (abort && *abort) return;
  __shared__ double v[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double s = 0.0;
  if (wave < 3) {
    for (int r = lane; r < nd; r += 64) s += dots_part[r * 3 + wave];
  } else if (!hilo) {
    for (int r = lane; r < nsse; r += 64) s += sse_part[r];
  }
  s = wave_sum(s);
  if (lane == 0) v[wave] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double sse = hilo ? (double(hilo[0]) + double(hilo[1])) : v[3];
    scal[SC_TGG] = v[0];
    scal[SC_TGP] = v[1];
    scal[SC_WW] = v[2];
    scal[SC_SSE] = sse;
    double loss = 0.5 * sse * inv_scale;
    if (lambda != 0.0) loss += 0.5 * lambda * v[2];
    scal[SC_LOSS] = loss;
  }
}

void eval_tail(hipStream_t s, const double *dots_part, int nd, const double *sse_part, int nsse, const float *hilo,
               double inv_scale, double lambda, double *scal, const int *abort) {
  hipLaunchKernelGGL(eval_tail_kernel, dim3(1), dim3(256), 0, s, dots_part, nd, sse_part, nsse, hilo, inv_scale,
                     lambda, scal, abort);
  LBF_KERNEL_CHECK();
}

// Data-parallel: reduce this rank's SSE partials and store them as an fp32 (hi, lo) pair behind the
// gradient, so one all-reduce of [grad | hi | lo] carries the loss with ~fp64 accuracy (sse_pack_body).
__global__ __launch_bounds__(64) void sse_pack_kernel(const double *sse_part, int nsse, float *hilo,
                                                      const int *abort) {
  if (abort && *abort) return;
  sse_pack_body(sse_part, nsse, hilo, threadIdx.x);
}

void sse_pack(hipStream_t s, const double *sse_part, int nsse, float *hilo, const int *abort) {
  hipLaunchKernelGGL(sse_pack_kernel, dim3(1), dim3(64), 0, s, sse_part, nsse, hilo, abort);
  LBF_KERNEL_CHECK();
}

// Acceptance test of the first line-search trial, evaluated exactly as the host would (no FMA
// contraction, same precision): Wolfe in fp64 (full_batch_minimizer.hpp:136-152), Armijo in fp32
// (lbfgs.cuh:159-163). Convergence uses the next iteration's entry test (lbfgs.hpp:42, lbfgs.cuh:143).
__global__ __launch_bounds__(64) void ls_ctl_kernel(const LsCtlArgs a) {
  if (threadIdx.x != 0 || *a.abort) return;
  double *sc = a.scal;
  const double fn = sc[SC_LOSS], gfo = sc[SC_GTP], gnp = sc[SC_TGP], tgg = sc[SC_TGG];
  bool ok, conv;
  if (!a.armijo) {
    const double fold = a.host_fold ? a.fold : sc[SC_FOLD];
    ok = a.first || (!(fn > __dadd_rn(fold, __dmul_rn(__dmul_rn(a.c1, a.alpha), gfo))) && !(gnp < __dmul_rn(a.c2, gfo)));
    conv = sqrt(tgg) < a.tol;
    if (ok) sc[SC_FOLD] = fn;
  } else {
    const float foldf = a.host_fold ? a.foldf : float(sc[SC_FOLDF]);
    const float lnew = float(fn), gdp = float(gfo);
    ok = lnew <= __fadd_rn(foldf, __fmul_rn(__fmul_rn(float(a.c1), a.alphaf), gdp));
    conv = float(sqrt(tgg)) < float(a.tol);
    if (ok) sc[SC_FOLDF] = double(lnew);
  }
  const int status = !ok ? SPEC_REJECT : (conv ? SPEC_CONVERGED : SPEC_ACCEPT);
  if (status != SPEC_ACCEPT) *a.abort = 1;
  // The record lives in host memory. Every field is stored write-through (system-scope relaxed
  // atomic stores: sc0 sc1, no cache write-back), the payload is acknowledged before the sequence word
  // is stored, so a host that sees seq sees the payload. (A system-scope release fence would write
  // back the whole L2 - microseconds for nothing here.)
  SpecRecord *r = a.rec;
  const double alpha0 = sc[SC_ALPHA0], accept_prev = sc[SC_ACCEPT];
  __hip_atomic_store(&r->loss, fn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&r->tgg, tgg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&r->alpha0, alpha0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&r->accept_prev, accept_prev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&r->status, status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(&r->seq, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

void ls_ctl(hipStream_t s, const LsCtlArgs &a) {
  hipLaunchKernelGGL(ls_ctl_kernel, dim3(1), dim3(64), 0, s, a);
  LBF_KERNEL_CHECK();
}

} // namespace lbf

#ifdef LBF_KTRACE
extern "C" int lbf_dbg_ktrace(unsigned long long *host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(lbf::lbf_kt_buf), size_t(n) * 8) == hipSuccess ? 0 : 1;
}
#endif
