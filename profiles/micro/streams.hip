// History-sweep read micro-benchmark (gfx950): what read rate can a k-vector linear combination reach?
//   hipcc --offload-arch=gfx950 -O3 streams.hip -o streams && ./streams
// k = 100 vectors of n = 10,489,857 floats (the cfg-5 history at m = 50, 4.2 GB):
//   contig   one contiguous 4.2 GB read, float4 per lane, sum reduction (ceiling)
//   sep      the combine pattern: each lane reads 16 B of every vector (separate n-vectors), fp64 acc
//   sep_nt   the same with nontemporal loads
//   blocked  history interleaved by 1024-float chunks: [n/1024][k][1024] (each block reads one
//            contiguous k*4 KB region)
#include <hip/hip_runtime.h>

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

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void contig_k(const f32x4 *p, long long n4, float *out) {
  double acc = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const f32x4 v = p[i];
    acc += double(v[0]) + double(v[1]) + double(v[2]) + double(v[3]);
  }
  if (acc == 123.456) out[0] = float(acc);
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void sep_k(const float *H, long long ld, int k, const double *c, float *out,
                                              long long n) {
  const long long e = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (e + 3 >= n) return;
  double acc[4] = {0, 0, 0, 0};
  int i = 0;
  for (; i + U <= k; i += U) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const f32x4 *p = reinterpret_cast<const f32x4 *>(H + (long long)(i + u) * ld + e);
      v[u] = NT ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] += c[i + u] * double(v[u][j]);
  }
  f32x4 d;
  for (int j = 0; j < 4; ++j) d[j] = float(acc[j]);
  *reinterpret_cast<f32x4 *>(out + e) = d;
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void sep_gs_k(const float *H, long long ld, int k, const double *c, float *out,
                                                 long long n) {
  for (long long e = ((long long)blockIdx.x * 256 + threadIdx.x) * 4; e + 3 < n; e += (long long)gridDim.x * 1024) {
    double acc[4] = {0, 0, 0, 0};
    int i = 0;
    for (; i + U <= k; i += U) {
      f32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const f32x4 *p = reinterpret_cast<const f32x4 *>(H + (long long)(i + u) * ld + e);
        v[u] = NT ? __builtin_nontemporal_load(p) : *p;
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] += c[i + u] * double(v[u][j]);
    }
    f32x4 d;
    for (int j = 0; j < 4; ++j) d[j] = float(acc[j]);
    *reinterpret_cast<f32x4 *>(out + e) = d;
  }
}

__global__ __launch_bounds__(256) void contig_nt_k(const f32x4 *p, long long n4, float *out) {
  double acc = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const f32x4 v = __builtin_nontemporal_load(p + i);
    acc += double(v[0]) + double(v[1]) + double(v[2]) + double(v[3]);
  }
  if (acc == 123.456) out[0] = float(acc);
}

// wave-per-vector combine: a 256-thread block owns a chunk of C floats; wave w accumulates vectors
// w, w+4, ... (each wave streams C*4 contiguous bytes of one vector at a time, nt loads), then the four
// wave sums are added in a fixed order through LDS.
template <int C, int VU>
__global__ __launch_bounds__(256) void wpv_k(const float *H, long long ld, int k, const double *c, float *out,
                                              long long n) {
  constexpr int Q = C / 256; // f32x4 per lane per vector
  __shared__ double red[3][C];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long e0 = (long long)blockIdx.x * C;
  double acc[4 * Q];
#pragma unroll
  for (int q = 0; q < 4 * Q; ++q) acc[q] = 0.0;
  for (int v0 = wave; v0 < k; v0 += 4 * VU) {
    f32x4 x[VU][Q];
#pragma unroll
    for (int u = 0; u < VU; ++u)
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int v = v0 + 4 * u;
        const long long e = e0 + (q * 64 + lane) * 4;
        x[u][q] = (v < k && e + 3 < n) ? __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(H + (long long)v * ld + e))
                                       : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
    for (int u = 0; u < VU; ++u) {
      const int v = v0 + 4 * u;
      if (v < k) {
        const double cv = c[v];
#pragma unroll
        for (int q = 0; q < Q; ++q)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[4 * q + j] += cv * double(x[u][q][j]);
      }
    }
  }
  if (wave > 0)
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[wave - 1][(q * 64 + lane) * 4 + j] = acc[4 * q + j];
  __syncthreads();
  if (wave == 0)
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const long long e = e0 + (q * 64 + lane) * 4;
      f32x4 d;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = (q * 64 + lane) * 4 + j;
        d[j] = float(((acc[4 * q + j] + red[0][i]) + red[1][i]) + red[2][i]);
      }
      if (e + 3 < n) *reinterpret_cast<f32x4 *>(out + e) = d;
    }
}

// blocked: chunk b of 1024 floats; element (vec i, pos e) at ((b*k + i)*1024 + e%1024)
template <int U>
__global__ __launch_bounds__(256) void blocked_k(const float *H, int k, const double *c, float *out, long long n) {
  const long long b = blockIdx.x;
  const long long e = b * 1024 + threadIdx.x * 4;
  if (e + 3 >= n) return;
  const float *base = H + b * (long long)k * 1024 + threadIdx.x * 4;
  double acc[4] = {0, 0, 0, 0};
  int i = 0;
  for (; i + U <= k; i += U) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const f32x4 *>(base + (long long)(i + u) * 1024);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] += c[i + u] * double(v[u][j]);
  }
  f32x4 d;
  for (int j = 0; j < 4; ++j) d[j] = float(acc[j]);
  *reinterpret_cast<f32x4 *>(out + e) = d;
}

int main() {
  const long long n = 10489857, ld = (n + 1023) / 1024 * 1024;
  const int k = 100;
  const size_t bytes = size_t(k) * ld * sizeof(float);
  float *H, *out, *flush;
  double *c;
  CK(hipMalloc(&H, bytes));
  CK(hipMalloc(&out, size_t(ld) * 4));
  CK(hipMalloc(&flush, size_t(512) << 20));
  CK(hipMalloc(&c, k * sizeof(double)));
  CK(hipMemset(H, 0, bytes));
  std::vector<double> hc(k, 0.5);
  CK(hipMemcpy(c, hc.data(), k * sizeof(double), hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const long long nread = (long long)k * n * 4;
  bool dirty = true;
  auto timeit = [&](const char *name, auto launch, double rbytes) -> int {
    float best = 1e30f, sum = 0.f;
    for (int r = 0; r < 6; ++r) {
      if (dirty) CK(hipMemsetAsync(flush, r, size_t(512) << 20)); // evict the caches (dirty lines)
      else hipLaunchKernelGGL(contig_k, dim3(2048), dim3(256), 0, 0, (const f32x4 *)flush, (512LL << 20) / 16, out);
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (r > 0) {
        best = ms < best ? ms : best;
        sum += ms;
      }
    }
    printf("%-14s best %8.1f us  %6.0f GB/s   avg %8.1f us  %6.0f GB/s\n", name, best * 1e3, rbytes / best / 1e6,
           sum / 5 * 1e3, rbytes / (sum / 5) / 1e6);
    return 0;
  };
  const unsigned g4 = unsigned((n / 4 + 255) / 256);
  timeit("contig", [&] { hipLaunchKernelGGL(contig_k, dim3(8192), dim3(256), 0, 0, (const f32x4 *)H, (long long)k * ld / 4, out); },
         double(k) * ld * 4);
  timeit("contig_2048", [&] { hipLaunchKernelGGL(contig_k, dim3(2048), dim3(256), 0, 0, (const f32x4 *)H, (long long)k * ld / 4, out); },
         double(k) * ld * 4);
  timeit("sep_u1", [&] { hipLaunchKernelGGL((sep_k<1, false>), dim3(g4), dim3(256), 0, 0, H, ld, k, c, out, n); }, nread);
  timeit("sep_u4", [&] { hipLaunchKernelGGL((sep_k<4, false>), dim3(g4), dim3(256), 0, 0, H, ld, k, c, out, n); }, nread);
  timeit("sep_u8", [&] { hipLaunchKernelGGL((sep_k<8, false>), dim3(g4), dim3(256), 0, 0, H, ld, k, c, out, n); }, nread);
  timeit("sep_u4_nt", [&] { hipLaunchKernelGGL((sep_k<4, true>), dim3(g4), dim3(256), 0, 0, H, ld, k, c, out, n); }, nread);
  timeit("sep_u8_nt", [&] { hipLaunchKernelGGL((sep_k<8, true>), dim3(g4), dim3(256), 0, 0, H, ld, k, c, out, n); }, nread);
  const unsigned gb = unsigned(ld / 1024);
  timeit("blocked_u4", [&] { hipLaunchKernelGGL((blocked_k<4>), dim3(gb), dim3(256), 0, 0, H, k, c, out, n); }, nread);
  timeit("blocked_u8", [&] { hipLaunchKernelGGL((blocked_k<8>), dim3(gb), dim3(256), 0, 0, H, k, c, out, n); }, nread);
  timeit("contig_nt_2048", [&] { hipLaunchKernelGGL(contig_nt_k, dim3(2048), dim3(256), 0, 0, (const f32x4 *)H, (long long)k * ld / 4, out); },
         double(k) * ld * 4);
  for (int gs : {1024, 2048, 4096}) {
    char nm[64];
    snprintf(nm, 64, "sep_gs%d_u4_nt", gs);
    timeit(nm, [&] { hipLaunchKernelGGL((sep_gs_k<4, true>), dim3(gs), dim3(256), 0, 0, H, ld, k, c, out, n); }, nread);
    snprintf(nm, 64, "sep_gs%d_u8_nt", gs);
    timeit(nm, [&] { hipLaunchKernelGGL((sep_gs_k<8, true>), dim3(gs), dim3(256), 0, 0, H, ld, k, c, out, n); }, nread);
    snprintf(nm, 64, "sep_gs%d_u4", gs);
    timeit(nm, [&] { hipLaunchKernelGGL((sep_gs_k<4, false>), dim3(gs), dim3(256), 0, 0, H, ld, k, c, out, n); }, nread);
  }
  timeit("wpv1024_v1", [&] { hipLaunchKernelGGL((wpv_k<1024, 1>), dim3(unsigned(ld / 1024)), dim3(256), 0, 0, H, ld, k, c, out, n); }, nread);
  timeit("wpv1024_v2", [&] { hipLaunchKernelGGL((wpv_k<1024, 2>), dim3(unsigned(ld / 1024)), dim3(256), 0, 0, H, ld, k, c, out, n); }, nread);
  timeit("wpv2048_v1", [&] { hipLaunchKernelGGL((wpv_k<2048, 1>), dim3(unsigned(ld / 2048 + 1)), dim3(256), 0, 0, H, ld, k, c, out, n); }, nread);
  timeit("wpv2048_v2", [&] { hipLaunchKernelGGL((wpv_k<2048, 2>), dim3(unsigned(ld / 2048 + 1)), dim3(256), 0, 0, H, ld, k, c, out, n); }, nread);
  // k = 20 (m = 10)
  const long long nread20 = 20LL * n * 4;
  timeit("sep_u4_k20", [&] { hipLaunchKernelGGL((sep_k<4, false>), dim3(g4), dim3(256), 0, 0, H, ld, 20, c, out, n); }, nread20);
  timeit("sep_u4nt_k20", [&] { hipLaunchKernelGGL((sep_k<4, true>), dim3(g4), dim3(256), 0, 0, H, ld, 20, c, out, n); }, nread20);
  timeit("blocked_u4_k20", [&] { hipLaunchKernelGGL((blocked_k<4>), dim3(gb), dim3(256), 0, 0, H, 20, c, out, n); }, nread20);
  if (dirty) {
    dirty = false;
    printf("---- clean flush (read 512 MB) ----\n");
    timeit("contig_2048", [&] { hipLaunchKernelGGL(contig_k, dim3(2048), dim3(256), 0, 0, (const f32x4 *)H, (long long)k * ld / 4, out); },
           double(k) * ld * 4);
    timeit("sep_u4", [&] { hipLaunchKernelGGL((sep_k<4, false>), dim3(g4), dim3(256), 0, 0, H, ld, k, c, out, n); }, nread);
    timeit("sep_u4_nt", [&] { hipLaunchKernelGGL((sep_k<4, true>), dim3(g4), dim3(256), 0, 0, H, ld, k, c, out, n); }, nread);
    timeit("sep_gs2048_u4_nt", [&] { hipLaunchKernelGGL((sep_gs_k<4, true>), dim3(2048), dim3(256), 0, 0, H, ld, k, c, out, n); }, nread);
    timeit("sep_gs2048_u4", [&] { hipLaunchKernelGGL((sep_gs_k<4, false>), dim3(2048), dim3(256), 0, 0, H, ld, k, c, out, n); }, nread);
    timeit("sep_u8_nt", [&] { hipLaunchKernelGGL((sep_k<8, true>), dim3(g4), dim3(256), 0, 0, H, ld, k, c, out, n); }, nread);
    timeit("wpv1024_v2", [&] { hipLaunchKernelGGL((wpv_k<1024, 2>), dim3(unsigned(ld / 1024)), dim3(256), 0, 0, H, ld, k, c, out, n); }, nread);
    timeit("wpv2048_v1", [&] { hipLaunchKernelGGL((wpv_k<2048, 1>), dim3(unsigned(ld / 2048 + 1)), dim3(256), 0, 0, H, ld, k, c, out, n); }, nread);
    timeit("wpv1024_v2_k20", [&] { hipLaunchKernelGGL((wpv_k<1024, 2>), dim3(unsigned(ld / 1024)), dim3(256), 0, 0, H, ld, 20, c, out, n); }, nread20);
    timeit("sep_u4_k20", [&] { hipLaunchKernelGGL((sep_k<4, false>), dim3(g4), dim3(256), 0, 0, H, ld, 20, c, out, n); }, nread20);
    timeit("sep_u4nt_k20", [&] { hipLaunchKernelGGL((sep_k<4, true>), dim3(g4), dim3(256), 0, 0, H, ld, 20, c, out, n); }, nread20);
    timeit("sep_gs2048_u4nt_k20", [&] { hipLaunchKernelGGL((sep_gs_k<4, true>), dim3(2048), dim3(256), 0, 0, H, ld, 20, c, out, n); }, nread20);
  }
  return 0;
}
