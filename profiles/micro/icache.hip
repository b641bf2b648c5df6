// Instruction-fetch cost of straight-line code in a single-block kernel (the optimizer-tail shape):
// N scalar adds unrolled (4 B each) vs the same count in a 64-instruction loop, each launch timed
// with s_memrealtime inside the kernel, after an L2/MALL-thrashing stream and back to back.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define A4 "s_add_u32 s8, s8, 1\n s_add_u32 s9, s9, 1\n s_add_u32 s10, s10, 1\n s_add_u32 s11, s11, 1\n"
#define A16 A4 A4 A4 A4
#define A64 A16 A16 A16 A16
#define A256 A64 A64 A64 A64
#define A1K A256 A256 A256 A256

__global__ void straight(unsigned long long *out) {
  unsigned long long t0 = wall_clock64();
  asm volatile(A1K A1K A1K A1K ::: "s8", "s9", "s10", "s11");
  unsigned long long t1 = wall_clock64();
  if (threadIdx.x == 0) out[0] = t1 - t0;
}
__global__ void looped(unsigned long long *out) {
  unsigned long long t0 = wall_clock64();
  for (int i = 0; i < 64; ++i) asm volatile(A64 ::: "s8", "s9", "s10", "s11");
  unsigned long long t1 = wall_clock64();
  if (threadIdx.x == 0) out[0] = t1 - t0;
}
__global__ void thrash(const float4 *in, float4 *out, size_t n) {
  float4 acc = {0, 0, 0, 0};
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) {
    float4 v = in[i];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  if (acc.x == 123.f) out[0] = acc;
}

int main() {
  unsigned long long *d, h;
  hipMalloc(&d, 64);
  size_t n = (size_t(1) << 30) / 16;
  float4 *buf, *o;
  hipMalloc(&buf, n * 16);
  hipMalloc(&o, 64);
  hipMemset(buf, 0, n * 16);
  auto run = [&](const char *name, void (*k)(unsigned long long *), bool flush) {
    double s = 0;
    for (int r = 0; r < 6; ++r) {
      if (flush) hipLaunchKernelGGL(thrash, dim3(2048), dim3(256), 0, 0, buf, o, n);
      hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
      hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
      if (r) s += h / 100.0;
    }
    printf("%-10s %-8s %.2f us per launch (4096 SALU ops)\n", name, flush ? "flushed" : "warm", s / 5);
  };
  run("straight", straight, true);
  run("looped", looped, true);
  run("straight", straight, false);
  run("looped", looped, false);
  return 0;
}
