// Dependent-load round trip on a 1-wave kernel: pointer chase over a buffer that is either
// untouched since long ago, or rewritten by a full-grid kernel launched just before.
//   hipcc --offload-arch=gfx950 -O3 chase.hip -o chase && ./chase
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void init_k(int *p, int n, int stride) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = (i + stride) % n;
}
__global__ void chase_k(const int *p, int hops, int *out) {
  int j = 0;
  for (int h = 0; h < hops; ++h) j = p[j];
  if (threadIdx.x == 0) *out = j;
}
__global__ void chase_volatile_k(const int *p, int hops, int *out) { // glc: bypass L1/L0
  int j = 0;
  for (int h = 0; h < hops; ++h) j = __hip_atomic_load(p + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x == 0) *out = j;
}

int main() {
  const int n = 1 << 20, stride = 4099;
  int *p, *out;
  hipMalloc(&p, n * 4);
  hipMalloc(&out, 64);
  hipStream_t s;
  hipStreamCreate(&s);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(init_k, n / 256, 256, 0, s, p, n, stride);
  const int R = 200;
  auto time = [&](const char *name, auto body) {
    for (int i = 0; i < 10; ++i) body();
    hipEventRecord(a, s);
    for (int i = 0; i < R; ++i) body();
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-60s %8.2f us/iter\n", name, ms * 1e3f / R);
  };
  for (int hops : {1, 10, 40}) {
    char nm[128];
    snprintf(nm, sizeof nm, "chase %d hops, static buffer", hops);
    time(nm, [&] { hipLaunchKernelGGL(chase_k, 1, 64, 0, s, p, hops, out); });
    snprintf(nm, sizeof nm, "chase %d hops (agent-scope loads), static buffer", hops);
    time(nm, [&] { hipLaunchKernelGGL(chase_volatile_k, 1, 64, 0, s, p, hops, out); });
    snprintf(nm, sizeof nm, "rewrite 4 MB (grid) + chase %d hops", hops);
    time(nm, [&] {
      hipLaunchKernelGGL(init_k, n / 256, 256, 0, s, p, n, stride);
      hipLaunchKernelGGL(chase_k, 1, 64, 0, s, p, hops, out);
    });
  }
  time("rewrite 4 MB (grid) alone", [&] { hipLaunchKernelGGL(init_k, n / 256, 256, 0, s, p, n, stride); });
  return 0;
}
