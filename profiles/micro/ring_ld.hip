// History-ring layout micro-benchmark (gfx950): does the slot stride of the (s, y) ring change the rate of the
// combine sweep's many-stream read (2k vectors, 16 B per lane of each, fp64 accumulate, grid-stride over the
// resident grid, nontemporal loads: vec_kernels.hip combine_kernel<8, true>) and of the Gram sweep's pattern
// (one wave per vector over a 4096-float chunk, 4 quads in flight)?
//   hipcc --offload-arch=gfx950 -O3 ring_ld.hip -o ring_ld && ./ring_ld
// n = 10,489,857 (cfg 5), k = 100 vectors (m = 50). Strides: round4(n) (the engine's), + 64 / 256 / 1024 / 4160
// floats, and rounded up to 2 MiB (+ 4 KiB).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                                                \
  do {                                                                                                       \
    hipError_t e_ = (x);                                                                                     \
    if (e_ != hipSuccess) {                                                                                  \
      printf("%s line %d\n", hipGetErrorString(e_), __LINE__);                                               \
      return 1;                                                                                              \
    }                                                                                                        \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void comb_k(const float *H, long long ld, int k, const double *c, float *out,
                                              long long n) {
  __shared__ double cs[128];
  for (int i = threadIdx.x; i < k; i += 256) cs[i] = c[i];
  __syncthreads();
  const long long stride = (long long)gridDim.x * 256 * 4;
  for (long long e = ((long long)blockIdx.x * 256 + threadIdx.x) * 4; e + 3 < n; e += stride) {
    double acc[4] = {0, 0, 0, 0};
    for (int i = 0; i + U <= k; i += U) {
      f32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(H + (long long)(i + u) * ld + e));
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] += cs[i + u] * double(v[u][j]);
    }
    f32x4 d;
    for (int j = 0; j < 4; ++j) d[j] = float(acc[j]);
    *reinterpret_cast<f32x4 *>(out + e) = d;
  }
}

// Gram pattern: a workgroup of 8 waves owns a 4096-float chunk; wave w streams vectors w, w + 8, ... of it, V vectors
// at a time with U of each vector's 16 quads per lane in flight (the engine's gram_kernel: V = 1, U = 4), dots
// against one LDS vector, a shuffle sum per vector.
template <int U, int V>
__global__ __launch_bounds__(512) void gram_k(const float *H, long long ld, int k, double *out, long long n) {
  __shared__ float g[4096];
  const long long e0 = (long long)blockIdx.x * 4096;
  for (int i = threadIdx.x; i < 4096; i += 512) g[i] = 1.0f + 1e-3f * float(i);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int v0 = wave; v0 < k; v0 += 8 * V) {
    double s[V];
#pragma unroll
    for (int q = 0; q < V; ++q) s[q] = 0.0;
    for (int i0 = lane * 4; i0 < 4096; i0 += 256 * U) {
      f32x4 x[V][U];
#pragma unroll
      for (int q = 0; q < V; ++q) {
        const int v = min(v0 + 8 * q, k - 1);
        const float *Vp = H + (long long)v * ld + e0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long ee = e0 + i0 + 256 * u;
          x[q][u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(Vp + (ee + 3 < n ? i0 + 256 * u : 0)));
        }
      }
#pragma unroll
      for (int q = 0; q < V; ++q)
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int j = 0; j < 4; ++j) s[q] += double(x[q][u][j]) * double(g[i0 + 256 * u + j]);
    }
#pragma unroll
    for (int q = 0; q < V; ++q) {
      double t = s[q];
      for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
      if (lane == 0 && v0 + 8 * q < k) out[(long long)blockIdx.x * 128 + v0 + 8 * q] = t;
    }
  }
}

// The engine's Gram sweep arithmetic on the same pattern: three fp32 vectors (s, y, g) of the chunk in LDS (48 KB:
// three workgroups per CU, as gram_kernel), three fp64 dots per history vector, V history vectors per pass sharing
// each LDS read, U quads of each in flight.
template <int U, int V, int TR = -1>
__global__ __launch_bounds__(512) void gram3_k(const float *H, long long ld, int k, double *out, long long n) {
  __shared__ float ls[4096], ly[4096], lg[4096];
  const long long e0 = (long long)blockIdx.x * 4096;
  for (int i = threadIdx.x; i < 4096; i += 512) {
    ls[i] = 1.0f + 1e-3f * float(i);
    ly[i] = 2.0f - 1e-3f * float(i);
    lg[i] = 0.5f + 1e-4f * float(i);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int v0 = wave; v0 < k; v0 += 8 * V) {
    double ds[V], dy[V], dg[V];
#pragma unroll
    for (int q = 0; q < V; ++q) ds[q] = dy[q] = dg[q] = 0.0;
    for (int i0 = lane * 4; i0 < 4096; i0 += 256 * U) {
      f32x4 x[V][U];
#pragma unroll
      for (int q = 0; q < V; ++q) {
        const int v = min(v0 + 8 * q, k - 1);
        const float *Vp = H + (long long)v * ld + e0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long ee = e0 + i0 + 256 * u;
          x[q][u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(Vp + (ee + 3 < n ? i0 + 256 * u : 0)));
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const f32x4 s4 = *reinterpret_cast<const f32x4 *>(ls + i0 + 256 * u);
        const f32x4 y4 = *reinterpret_cast<const f32x4 *>(ly + i0 + 256 * u);
        const f32x4 g4 = *reinterpret_cast<const f32x4 *>(lg + i0 + 256 * u);
#pragma unroll
        for (int q = 0; q < V; ++q)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const double xv = x[q][u][j];
            ds[q] += xv * double(s4[j]);
            dy[q] += xv * double(y4[j]);
            dg[q] += xv * double(g4[j]);
          }
      }
    }
#pragma unroll
    for (int q = 0; q < V; ++q) {
      if (TR < 0) {
        double t = ds[q] + 2.0 * dy[q] + 3.0 * dg[q];
        for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
        if (lane == 0 && v0 + 8 * q < k) out[(long long)blockIdx.x * 128 + v0 + 8 * q] = t;
      } else { // the engine's three partials per vector: transposed [col][block] (TR = 1) or [block][col] (TR = 0)
        double d3[3] = {ds[q], dy[q], dg[q]};
        for (int c = 0; c < 3; ++c)
          for (int o = 32; o > 0; o >>= 1) d3[c] += __shfl_xor(d3[c], o);
        const int col = 3 * (v0 + 8 * q);
        if (lane == 0 && v0 + 8 * q < k)
          for (int c = 0; c < 3; ++c)
            out[TR ? (long long)(col + c) * gridDim.x + blockIdx.x : (long long)blockIdx.x * 384 + col + c] = d3[c];
      }
    }
  }
}

// gram3 with the engine's first phase: per chunk the new vectors s = x - xp, y = g - gp and g formed from five
// 16-B operand streams into LDS, s and y written to a ring slot, g to g_out, six self dots reduced over the block,
// then the history phase (gram3_k<4, 1, 0>'s, row-major partials).
template <int VAR> // 0: the engine's phase 1; 1: without its three global stores; 2: without the block reduction;
                   // 3: the new vectors read from three streams (s, y, g precomputed: a split sweep's second kernel)
__global__ __launch_bounds__(512) void gram3p_k(const float *H, long long ld, int k, double *out, long long n,
                                                const float *x, const float *xp, const float *g, const float *gp,
                                                float *sw, float *yw, float *gout) {
  __shared__ __attribute__((aligned(16))) float ls[4096], ly[4096], lg[4096];
  __shared__ double red[8][6];
  const long long e0 = (long long)blockIdx.x * 4096;
  double self[6] = {0, 0, 0, 0, 0, 0};
  const int nq = int(min(4096LL, n - e0) >> 2);
  for (int q0 = threadIdx.x; q0 < nq; q0 += 1024) {
    f32x4 op[2][5];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int q = min(q0 + u * 512, nq - 1);
      const long long e = e0 + 4LL * q;
      const float *src[5] = {x, xp, g, gp, g};
      if (VAR == 3) {
        src[0] = sw;
        src[2] = yw;
      }
#pragma unroll
      for (int j = 0; j < 5; ++j)
        if (VAR != 3 || j == 0 || j == 2 || j == 4) op[u][j] = *reinterpret_cast<const f32x4 *>(src[j] + e);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int q = q0 + u * 512;
      if (q >= nq) break;
      const f32x4 s4 = VAR == 3 ? op[u][0] : op[u][0] - op[u][1], y4 = VAR == 3 ? op[u][2] : op[u][2] - op[u][3];
      const f32x4 g4 = op[u][4];
      *reinterpret_cast<f32x4 *>(ls + 4 * q) = s4;
      *reinterpret_cast<f32x4 *>(ly + 4 * q) = y4;
      *reinterpret_cast<f32x4 *>(lg + 4 * q) = g4;
      if (VAR == 0 || VAR == 2) {
        *reinterpret_cast<f32x4 *>(sw + e0 + 4 * q) = s4;
        *reinterpret_cast<f32x4 *>(yw + e0 + 4 * q) = y4;
        *reinterpret_cast<f32x4 *>(gout + e0 + 4 * q) = g4;
      }
      for (int c = 0; c < 4; ++c) {
        const double sv = s4[c], yv = y4[c], gv = g4[c];
        self[0] += sv * sv; self[1] += sv * yv; self[2] += yv * yv;
        self[3] += gv * sv; self[4] += gv * yv; self[5] += gv * gv;
      }
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (VAR != 2 && VAR != 3) {
    for (int j = 0; j < 6; ++j) {
      double t = self[j];
      for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
      if (lane == 0) red[wave][j] = t;
    }
    __syncthreads();
    if (threadIdx.x < 6) {
      double t = 0;
      for (int w = 0; w < 8; ++w) t += red[w][threadIdx.x];
      out[(long long)blockIdx.x * 384 + 300 + threadIdx.x] = t;
    }
  } else {
    __syncthreads();
    if (self[0] == 1234.5) out[0] = self[1] + self[2] + self[3] + self[4] + self[5]; // keep the products
  }
  for (int v0 = wave; v0 < k; v0 += 8) {
    double ds = 0, dy = 0, dg = 0;
    const float *Vp = H + (long long)v0 * ld + e0;
    for (int i0 = lane * 4; i0 < 4096; i0 += 1024) {
      f32x4 xv4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long long ee = e0 + i0 + 256 * u;
        xv4[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(Vp + (ee + 3 < n ? i0 + 256 * u : 0)));
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const f32x4 s4 = *reinterpret_cast<const f32x4 *>(ls + i0 + 256 * u);
        const f32x4 y4 = *reinterpret_cast<const f32x4 *>(ly + i0 + 256 * u);
        const f32x4 g4 = *reinterpret_cast<const f32x4 *>(lg + i0 + 256 * u);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const double xv = xv4[u][j];
          ds += xv * double(s4[j]);
          dy += xv * double(y4[j]);
          dg += xv * double(g4[j]);
        }
      }
    }
    double d3[3] = {ds, dy, dg};
    for (int c = 0; c < 3; ++c)
      for (int o = 32; o > 0; o >>= 1) d3[c] += __shfl_xor(d3[c], o);
    if (lane == 0)
      for (int c = 0; c < 3; ++c) out[(long long)blockIdx.x * 384 + 3 * v0 + c] = d3[c];
  }
}

// gram3p_k<0> as a persistent, software-pipelined sweep: a resident grid, each workgroup taking chunks
// blockIdx.x, blockIdx.x + gridDim.x, ...; the next chunk's four operand quads per thread are requested into
// registers before the current chunk's history phase, so phase 1 of the next chunk finds them landed.
__global__ __launch_bounds__(512) void gram3pp_k(const float *H, long long ld, int k, double *out, long long n,
                                                 const float *x, const float *xp, const float *g, const float *gp,
                                                 float *sw, float *yw, float *gout, int nch) {
  __shared__ __attribute__((aligned(16))) float ls[4096], ly[4096], lg[4096];
  __shared__ double red[8][6];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  f32x4 op[2][4];
  auto fetch = [&](int ch) {
    const long long e0 = (long long)ch * 4096;
    const int nq = int(min(4096LL, n - e0) >> 2);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int q = min(int(threadIdx.x) + u * 512, nq - 1);
      const long long e = e0 + 4LL * q;
      op[u][0] = *reinterpret_cast<const f32x4 *>(x + e);
      op[u][1] = *reinterpret_cast<const f32x4 *>(xp + e);
      op[u][2] = *reinterpret_cast<const f32x4 *>(g + e);
      op[u][3] = *reinterpret_cast<const f32x4 *>(gp + e);
    }
  };
  int ch = blockIdx.x;
  if (ch < nch) fetch(ch);
  for (; ch < nch; ch += gridDim.x) {
    const long long e0 = (long long)ch * 4096;
    const int nq = int(min(4096LL, n - e0) >> 2);
    double self[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int q = int(threadIdx.x) + u * 512;
      if (q >= nq) break;
      const f32x4 s4 = op[u][0] - op[u][1], y4 = op[u][2] - op[u][3], g4 = op[u][2];
      *reinterpret_cast<f32x4 *>(ls + 4 * q) = s4;
      *reinterpret_cast<f32x4 *>(ly + 4 * q) = y4;
      *reinterpret_cast<f32x4 *>(lg + 4 * q) = g4;
      *reinterpret_cast<f32x4 *>(sw + e0 + 4 * q) = s4;
      *reinterpret_cast<f32x4 *>(yw + e0 + 4 * q) = y4;
      *reinterpret_cast<f32x4 *>(gout + e0 + 4 * q) = g4;
      for (int c = 0; c < 4; ++c) {
        const double sv = s4[c], yv = y4[c], gv = g4[c];
        self[0] += sv * sv; self[1] += sv * yv; self[2] += yv * yv;
        self[3] += gv * sv; self[4] += gv * yv; self[5] += gv * gv;
      }
    }
    for (int j = 0; j < 6; ++j) {
      double t = self[j];
      for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
      if (lane == 0) red[wave][j] = t;
    }
    __syncthreads();
    if (threadIdx.x < 6) {
      double t = 0;
      for (int w = 0; w < 8; ++w) t += red[w][threadIdx.x];
      out[(long long)ch * 384 + 300 + threadIdx.x] = t;
    }
    if (ch + int(gridDim.x) < nch) fetch(ch + gridDim.x); // in flight during the history phase
    for (int v0 = wave; v0 < k; v0 += 8) {
      double ds = 0, dy = 0, dg = 0;
      const float *Vp = H + (long long)v0 * ld + e0;
      for (int i0 = lane * 4; i0 < 4096; i0 += 1024) {
        f32x4 xv4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const long long ee = e0 + i0 + 256 * u;
          xv4[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(Vp + (ee + 3 < n ? i0 + 256 * u : 0)));
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const f32x4 s4 = *reinterpret_cast<const f32x4 *>(ls + i0 + 256 * u);
          const f32x4 y4 = *reinterpret_cast<const f32x4 *>(ly + i0 + 256 * u);
          const f32x4 g4 = *reinterpret_cast<const f32x4 *>(lg + i0 + 256 * u);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const double xv = xv4[u][j];
            ds += xv * double(s4[j]);
            dy += xv * double(y4[j]);
            dg += xv * double(g4[j]);
          }
        }
      }
      double d3[3] = {ds, dy, dg};
      for (int c = 0; c < 3; ++c)
        for (int o = 32; o > 0; o >>= 1) d3[c] += __shfl_xor(d3[c], o);
      if (lane == 0)
        for (int c = 0; c < 3; ++c) out[(long long)ch * 384 + 3 * v0 + c] = d3[c];
    }
    __syncthreads(); // the LDS vectors are rewritten by the next chunk
  }
}

int main() {
  const long long n = 10489857, n4 = (n + 3) & ~3LL;
  const int k = 100;
  const long long pads[] = {0, 64, 256, 1024, 4160, -1, -2};
  int dev = 0, cus = 0, per = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, comb_k<8>, 256, 0));
  const long long maxld = ((n4 * 4 + (2 << 20) - 1) / (2 << 20)) * (2 << 20) / 4 + 1024;
  float *H = nullptr, *out = nullptr, *flush = nullptr;
  double *c = nullptr, *gout = nullptr;
  CK(hipMalloc(&H, size_t(maxld) * k * 4));
  CK(hipMalloc(&out, size_t(n4) * 4));
  CK(hipMalloc(&flush, size_t(512) << 20));
  CK(hipMalloc(&c, 128 * 8));
  const int nch = int((n + 4095) / 4096);
  CK(hipMalloc(&gout, size_t(nch) * 384 * 8));
  float *V5 = nullptr; // gram3p's operand and output vectors (x, xp, g, gp, s slot, y slot, g_out)
  CK(hipMalloc(&V5, size_t(7) * n4 * 4));
  CK(hipMemset(V5, 0, size_t(7) * n4 * 4));
  CK(hipMemset(H, 0, size_t(maxld) * k * 4));
  std::vector<double> hc(128, 0.01);
  CK(hipMemcpy(c, hc.data(), 128 * 8, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  printf("n = %lld, k = %d, combine grid %d x 256 (%d per CU), gram %d chunks\n", n, k, cus * per, per, nch);
  for (long long pad : pads) {
    long long ld = n4 + (pad > 0 ? pad : 0);
    if (pad == -1) ld = ((n4 * 4 + (2 << 20) - 1) / (2 << 20)) * (2 << 20) / 4;
    if (pad == -2) ld = ((n4 * 4 + (2 << 20) - 1) / (2 << 20)) * (2 << 20) / 4 + 1024;
    double bytes = double(k) * n * 4;
    const char *names[] = {"combine", "gram_u4v1", "gram_u8v1", "gram_u16v1", "gram_u8v2", "gram3_u4v1", "gram3_u4v2",
                           "gram3_u8v1", "gram3_tr1", "gram3_tr0", "gram3p", "gram3p_nost", "gram3p_nored",
                           "gram3p_split"};
    for (int kind = 0; kind < 14; ++kind) {
      if (kind > 1 && pad != 0 && pad != -2) continue; // the in-flight variants at two strides only
      float best = 1e30f, sum = 0.0f;
      // gram3p: + 4 operand reads and 3 writes (g read twice); without the stores + 4; split: + 3 reads
      bytes = double(k + (kind == 10 || kind == 12 ? 7 : (kind == 11 ? 4 : (kind == 13 ? 3 : 0)))) * n * 4;
      for (int it = 0; it < 6; ++it) {
        CK(hipMemset(flush, it, size_t(512) << 20)); // evict the Infinity Cache between runs
        CK(hipEventRecord(a));
        if (kind == 0) hipLaunchKernelGGL(comb_k<8>, dim3(cus * per), dim3(256), 0, 0, H, ld, k, c, out, n);
        else if (kind == 1) hipLaunchKernelGGL((gram_k<4, 1>), dim3(nch), dim3(512), 0, 0, H, ld, k, gout, n);
        else if (kind == 2) hipLaunchKernelGGL((gram_k<8, 1>), dim3(nch), dim3(512), 0, 0, H, ld, k, gout, n);
        else if (kind == 3) hipLaunchKernelGGL((gram_k<16, 1>), dim3(nch), dim3(512), 0, 0, H, ld, k, gout, n);
        else if (kind == 4) hipLaunchKernelGGL((gram_k<8, 2>), dim3(nch), dim3(512), 0, 0, H, ld, k, gout, n);
        else if (kind == 5) hipLaunchKernelGGL((gram3_k<4, 1>), dim3(nch), dim3(512), 0, 0, H, ld, k, gout, n);
        else if (kind == 6) hipLaunchKernelGGL((gram3_k<4, 2>), dim3(nch), dim3(512), 0, 0, H, ld, k, gout, n);
        else if (kind == 7) hipLaunchKernelGGL((gram3_k<8, 1>), dim3(nch), dim3(512), 0, 0, H, ld, k, gout, n);
        else if (kind == 8) hipLaunchKernelGGL((gram3_k<4, 1, 1>), dim3(nch), dim3(512), 0, 0, H, ld, k, gout, n);
        else if (kind == 9) hipLaunchKernelGGL((gram3_k<4, 1, 0>), dim3(nch), dim3(512), 0, 0, H, ld, k, gout, n);
        else if (kind == 10) hipLaunchKernelGGL(gram3p_k<0>, dim3(nch), dim3(512), 0, 0, H, ld, k, gout, n, V5, V5 + n4,
                                                V5 + 2 * n4, V5 + 3 * n4, V5 + 4 * n4, V5 + 5 * n4, V5 + 6 * n4);
        else if (kind == 11) hipLaunchKernelGGL(gram3p_k<1>, dim3(nch), dim3(512), 0, 0, H, ld, k, gout, n, V5, V5 + n4,
                                                V5 + 2 * n4, V5 + 3 * n4, V5 + 4 * n4, V5 + 5 * n4, V5 + 6 * n4);
        else if (kind == 12) hipLaunchKernelGGL(gram3p_k<2>, dim3(nch), dim3(512), 0, 0, H, ld, k, gout, n, V5, V5 + n4,
                                                V5 + 2 * n4, V5 + 3 * n4, V5 + 4 * n4, V5 + 5 * n4, V5 + 6 * n4);
        else hipLaunchKernelGGL(gram3p_k<3>, dim3(nch), dim3(512), 0, 0, H, ld, k, gout, n, V5, V5 + n4,
                                V5 + 2 * n4, V5 + 3 * n4, V5 + 4 * n4, V5 + 5 * n4, V5 + 6 * n4);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        if (it > 0) {
          best = ms < best ? ms : best;
          sum += ms;
        }
      }
      printf("%-10s ld = n4 %+6lld floats (%s)  best %7.1f us %6.0f GB/s  avg %7.1f us %6.0f GB/s\n",
             names[kind], ld - n4, pad == -1 ? "2 MiB" : (pad == -2 ? "2 MiB + 4 KiB" : "plain"),
             best * 1e3, bytes / best / 1e6, sum / 5 * 1e3, bytes / (sum / 5) / 1e6);
    }
  }
  // the fused sweep against its persistent, pipelined form, at m = 10 and m = 50 (k = 20, 100 history vectors)
  {
    int pp = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pp, gram3pp_k, 512, 0));
    for (int kk : {20, 100}) {
      const long long ld = n4;
      for (int kind = 0; kind < 4; ++kind) { // gram3p, gram3pp at 1x / 2x the resident grid, gram3p_split
        float best = 1e30f, sum = 0.0f;
        const double bytes = double(kk + (kind == 3 ? 3 : 7)) * n * 4;
        for (int it = 0; it < 6; ++it) {
          CK(hipMemset(flush, it, size_t(512) << 20));
          CK(hipEventRecord(a));
          if (kind == 0)
            hipLaunchKernelGGL(gram3p_k<0>, dim3(nch), dim3(512), 0, 0, H, ld, kk, gout, n, V5, V5 + n4, V5 + 2 * n4,
                               V5 + 3 * n4, V5 + 4 * n4, V5 + 5 * n4, V5 + 6 * n4);
          else if (kind == 3)
            hipLaunchKernelGGL(gram3p_k<3>, dim3(nch), dim3(512), 0, 0, H, ld, kk, gout, n, V5, V5 + n4, V5 + 2 * n4,
                               V5 + 3 * n4, V5 + 4 * n4, V5 + 5 * n4, V5 + 6 * n4);
          else
            hipLaunchKernelGGL(gram3pp_k, dim3(std::min(nch, cus * pp * kind)), dim3(512), 0, 0, H, ld, kk, gout, n, V5,
                               V5 + n4, V5 + 2 * n4, V5 + 3 * n4, V5 + 4 * n4, V5 + 5 * n4, V5 + 6 * n4, nch);
          CK(hipEventRecord(b));
          CK(hipEventSynchronize(b));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, a, b));
          if (it > 0) {
            best = ms < best ? ms : best;
            sum += ms;
          }
        }
        const char *nm[] = {"gram3p", "gram3pp_x1", "gram3pp_x2", "gram3p_split"};
        printf("k = %3d %-12s (%d per CU) best %7.1f us %6.0f GB/s  avg %7.1f us %6.0f GB/s\n", kk, nm[kind], pp,
               best * 1e3, bytes / best / 1e6, sum / 5 * 1e3, bytes / (sum / 5) / 1e6);
      }
    }
  }
  CK(hipFree(H));
  CK(hipFree(out));
  CK(hipFree(flush));
  CK(hipFree(c));
  CK(hipFree(gout));
  printf("done\n");
  return 0;
}
