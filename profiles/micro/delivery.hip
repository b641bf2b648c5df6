// Per-CU operand-delivery rates on gfx950 (round 5): how many bytes per cycle one CU pulls from an
// L2-resident region by LDS-DMA (global_load_lds_dwordx4), by 16-B register loads (global_load_dwordx4) and
// by 4-B register loads, with 4 or 8 waves per workgroup and 1 or 2 workgroups per CU, keeping D loads in
// flight per wave. Question: is the ~10-11 B/cycle/CU that the small-tile GEMMs move (32 x 128 forward,
// 64 x 64 dW; profiles/r02 gemm_small_tiles) a limit of the LDS-DMA path, or of the kernels' structure?
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 delivery.hip -o delivery && ./delivery
#include <hip/hip_runtime.h>

#include <cstdio>

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
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int REGION = 64 * 1024;     // bytes re-read by a workgroup (L2-resident after the first pass)
constexpr int ITERS = 4096;           // pieces (1 KiB per wave-instruction) per wave

template <int D> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D) : "memory"); }

// LDS-DMA: every wave streams 1-KiB pieces of the region into its own 8-slot LDS ring, D in flight.
template <int D, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void dma_kernel(const float *src, int shared, float *sink) {
  __shared__ __attribute__((aligned(16))) float ring[WAVES][8][256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const char *base = reinterpret_cast<const char *>(src) + (shared ? 0 : size_t(blockIdx.x) * REGION);
  for (int i = 0; i < ITERS; ++i) {
    const int piece = (i * WAVES + wave) % (REGION / 1024);
    const float *p = reinterpret_cast<const float *>(base + piece * 1024 + lane * 16);
    __builtin_amdgcn_global_load_lds((glb_void_t *)p, (lds_void_t *)&ring[wave][i & 7][0], 16, 0, 0);
    if (i >= D) vm_wait<D>();
  }
  vm_wait<0>();
  __syncthreads();
  if (threadIdx.x == 0) sink[blockIdx.x] = ring[0][0][0] + ring[WAVES - 1][7][255];
}

// 16-B register loads, D per batch in flight, summed (so the loads stay).
template <int D, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void reg16_kernel(const float *src, int shared, float *sink) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const char *base = reinterpret_cast<const char *>(src) + (shared ? 0 : size_t(blockIdx.x) * REGION);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < ITERS; i += D) {
    f32x4 v[D];
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int piece = ((i + u) * WAVES + wave) % (REGION / 1024);
      v[u] = *reinterpret_cast<const f32x4 *>(base + piece * 1024 + lane * 16);
    }
#pragma unroll
    for (int u = 0; u < D; ++u) acc += v[u];
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) sink[blockIdx.x] = 1.f;
}

// 4-B register loads (256 B per wave-instruction), D per batch.
template <int D, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void reg4_kernel(const float *src, int shared, float *sink) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const char *base = reinterpret_cast<const char *>(src) + (shared ? 0 : size_t(blockIdx.x) * REGION);
  float acc = 0.f;
  for (int i = 0; i < 4 * ITERS; i += D) {
    float v[D];
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int piece = ((i + u) * WAVES + wave) % (REGION / 256);
      v[u] = *reinterpret_cast<const float *>(base + piece * 256 + lane * 4);
    }
#pragma unroll
    for (int u = 0; u < D; ++u) acc += v[u];
  }
  if (acc == 12345.f) sink[blockIdx.x] = 1.f;
}

template <class K>
static double time_it(K kern, int blocks, int threads, const float *src, int shared, float *sink) {
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, src, shared, sink);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, 0);
  const int reps = 10;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, src, shared, sink);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms / reps * 1e-3;
}

template <int D, int WAVES>
static void row(const char *kind, int per_cu, const float *src, int shared, float *sink, int cus) {
  const int blocks = cus * per_cu, threads = 64 * WAVES;
  double s = 0;
  if (kind[0] == 'd') s = time_it(dma_kernel<D, WAVES>, blocks, threads, src, shared, sink);
  else if (kind[3] == '1') s = time_it(reg16_kernel<D, WAVES>, blocks, threads, src, shared, sink);
  else s = time_it(reg4_kernel<D, WAVES>, blocks, threads, src, shared, sink);
  const double bytes = double(blocks) * WAVES * double(ITERS) * 1024.0;
  const double per_cu_gbs = bytes / s / cus / 1e9;
  printf("%-6s waves %d  WG/CU %d  in-flight %2d  %s  %8.1f us  %7.1f GB/s per CU  %6.2f B/clk/CU @2.1GHz\n", kind,
         WAVES, per_cu, D, shared ? "shared region " : "own region   ", s * 1e6, per_cu_gbs, per_cu_gbs / 2.1);
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  float *src = nullptr, *sink = nullptr;
  CK(hipMalloc(&src, size_t(2 * cus) * REGION));
  CK(hipMemset(src, 0, size_t(2 * cus) * REGION));
  CK(hipMalloc(&sink, size_t(2 * cus) * sizeof(float)));
  printf("# %d CUs, %d KiB region per workgroup, %d KiB per wave per launch\n", cus, REGION / 1024, ITERS);
  for (int shared = 0; shared < 2; ++shared) {
    row<4, 4>("dma", 1, src, shared, sink, cus);
    row<8, 4>("dma", 1, src, shared, sink, cus);
    row<16, 4>("dma", 1, src, shared, sink, cus);
    row<8, 8>("dma", 1, src, shared, sink, cus);
    row<8, 4>("dma", 2, src, shared, sink, cus);
    row<8, 4>("reg16", 1, src, shared, sink, cus);
    row<16, 4>("reg16", 1, src, shared, sink, cus);
    row<8, 8>("reg16", 1, src, shared, sink, cus);
    row<8, 4>("reg16", 2, src, shared, sink, cus);
    row<16, 4>("reg4", 1, src, shared, sink, cus);
    row<16, 8>("reg4", 1, src, shared, sink, cus);
  }
  CK(hipDeviceSynchronize());
  printf("delivery ok\n");
  return 0;
}
