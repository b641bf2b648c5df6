// Launch-floor micro-benchmark (gfx950): back-to-back dependent launches on one stream.
//   hipcc --offload-arch=gfx950 -O3 launch_floor.hip -o launch_floor && ./launch_floor
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

__global__ void empty_k() {}
__global__ void write_k(double *p, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = double(i);
}
// one block sums n doubles (fixed per-thread rows, then a tree)
__global__ void onesum_k(const double *p, long long n, double *out) {
  __shared__ double ws[16];
  double s = 0.0;
  for (long long r = threadIdx.x; r < n; r += blockDim.x) s += p[r];
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double x = 0.0;
    for (int w = 0; w < int(blockDim.x >> 6); ++w) x += ws[w];
    *out = x;
  }
}

// one link of a dependent chain: every block reads the value the previous launch wrote and writes
// its successor (a true data dependency, as between the kernels of an evaluation)
__global__ void chain_k(double *p, int nb) {
  const double v = p[0];
  __syncthreads();
  if (threadIdx.x == 0) p[1 + blockIdx.x % 64] = v + 1.0;
  if (blockIdx.x == 0 && threadIdx.x == 0) p[0] = v + 1.0;
}

// one thread publishes a record to host-mapped coherent memory the way tail_fin does (system-scope
// relaxed stores, vmcnt(0), then the sequence word)
struct Rec { double a, b, c, d; int status, seq; };
__global__ void publish_k(Rec *r, int seq) {
  if (threadIdx.x == 0) {
    __hip_atomic_store(&r->a, 1.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&r->b, 2.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&r->c, 3.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&r->d, 4.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&r->status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&r->seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
// the same record in device memory
__global__ void publish_dev_k(Rec *r, int seq) {
  if (threadIdx.x == 0) {
    r->a = 1.0; r->b = 2.0; r->c = 3.0; r->d = 4.0; r->status = 1;
    __atomic_store_n(&r->seq, seq, __ATOMIC_RELAXED);
  }
}


int main() {
  setvbuf(stdout, nullptr, _IONBF, 0); // a crash keeps the lines printed so far
  double *buf, *out;
  const long long N = 1 << 22;
  CK(hipMalloc(&buf, N * 8));
  CK(hipMalloc(&out, 64));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t a, b, m;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventCreateWithFlags(&m, hipEventDisableTiming));
  const int R = 400;
  auto time = [&](const char *name, auto body) {
    for (int i = 0; i < 20; ++i) body();
    hipEventRecord(a, s);
    for (int i = 0; i < R; ++i) body();
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-58s %8.2f us/iter\n", name, ms * 1e3f / R);
  };
  time("empty<<<1,64>>>", [&] { hipLaunchKernelGGL(empty_k, 1, 64, 0, s); });
  time("empty<<<1024,256>>>", [&] { hipLaunchKernelGGL(empty_k, 1024, 256, 0, s); });
  time("empty + hipEventRecord(disable timing)", [&] {
    hipLaunchKernelGGL(empty_k, 1, 64, 0, s);
    hipEventRecord(m, s);
  });
  for (long long n : {2048LL, 8192LL}) {
    for (int th : {256, 1024}) {
      char nm[128];
      snprintf(nm, sizeof nm, "write %lld dbl (grid) + onesum<<<1,%d>>>", n, th);
      time(nm, [&] {
        hipLaunchKernelGGL(write_k, (unsigned)((n + 255) / 256), 256, 0, s, buf, n);
        hipLaunchKernelGGL(onesum_k, 1, th, 0, s, buf, n, out);
      });
    }
  }
  time("write 8192 dbl (grid) alone", [&] { hipLaunchKernelGGL(write_k, 32, 256, 0, s, buf, 8192LL); });
  time("write 32 MB (grid) alone", [&] { hipLaunchKernelGGL(write_k, (unsigned)(N / 256), 256, 0, s, buf, N); });
  time("write 32 MB + onesum 8192 <<<1,1024>>>", [&] {
    hipLaunchKernelGGL(write_k, (unsigned)(N / 256), 256, 0, s, buf, N);
    hipLaunchKernelGGL(onesum_k, 1, 1024, 0, s, buf, 8192LL, out);
  });
  // what a kernel that publishes to host-mapped memory costs its successor (tail_cols_fin -> combine)
  {
    Rec *hrec, *drec;
    CK(hipHostMalloc(reinterpret_cast<void **>(&hrec), sizeof(Rec), hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipMalloc(&drec, sizeof(Rec)));
    int seq = 0;
    time("empty<<<256,256>>> x3 (reference chain)", [&] {
      for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(empty_k, 256, 256, 0, s);
    });
    time("empty, publish_k (host-mapped record), empty", [&] {
      hipLaunchKernelGGL(empty_k, 256, 256, 0, s);
      hipLaunchKernelGGL(publish_k, 1, 64, 0, s, hrec, ++seq);
      hipLaunchKernelGGL(empty_k, 256, 256, 0, s);
    });
    time("empty, publish_dev_k (device record), empty", [&] {
      hipLaunchKernelGGL(empty_k, 256, 256, 0, s);
      hipLaunchKernelGGL(publish_dev_k, 1, 64, 0, s, drec, ++seq);
      hipLaunchKernelGGL(empty_k, 256, 256, 0, s);
    });
    CK(hipHostFree(hrec));
    CK(hipFree(drec));
  }
  // cross-stream hand-off per step: s2 waits for s's work, then s waits for s2's (the S-LBFGS twin's
  // pattern): with events, and with stream memory operations (write / wait on a device word)
  {
    hipStream_t s2;
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t e1, e2;
    CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
    unsigned *flag;
    CK(hipMalloc(&flag, 64));
    CK(hipMemset(flag, 0, 64));
    unsigned seq = 0;
    time("ping-pong s -> s2 -> s, events (per round trip)", [&] {
      hipLaunchKernelGGL(empty_k, 1, 64, 0, s);
      hipEventRecord(e1, s);
      hipStreamWaitEvent(s2, e1, 0);
      hipLaunchKernelGGL(empty_k, 1, 64, 0, s2);
      hipEventRecord(e2, s2);
      hipStreamWaitEvent(s, e2, 0);
    });
    time("ping-pong s -> s2 -> s, stream write/wait value", [&] {
      ++seq;
      hipLaunchKernelGGL(empty_k, 1, 64, 0, s);
      hipStreamWriteValue32(s, flag, 2 * seq, 0);
      hipStreamWaitValue32(s2, flag, 2 * seq, hipStreamWaitValueGte, 0xffffffffu);
      hipLaunchKernelGGL(empty_k, 1, 64, 0, s2);
      hipStreamWriteValue32(s2, flag + 16, 2 * seq, 0);
      hipStreamWaitValue32(s, flag + 16, 2 * seq, hipStreamWaitValueGte, 0xffffffffu);
    });
    time("two empty launches, one stream (reference)", [&] {
      hipLaunchKernelGGL(empty_k, 1, 64, 0, s);
      hipLaunchKernelGGL(empty_k, 1, 64, 0, s);
    });
    // teardown in dependency order: every event recorded on s2 and the word both streams wait on go before
    // s2 itself (round 3 left them, and s, a, b, m, buf, out, to the runtime's exit-time teardown)
    CK(hipStreamSynchronize(s));
    CK(hipStreamSynchronize(s2));
    CK(hipEventDestroy(e1));
    CK(hipEventDestroy(e2));
    CK(hipFree(flag));
    CK(hipStreamDestroy(s2));
  }
  // dependent chains of 10 launches at several grid sizes: eager, and the same chain as one hipGraph
  for (int nb : {1, 16, 64, 256, 1024}) {
    char nm[128];
    snprintf(nm, sizeof nm, "chain of 10 x chain_k<<<%d,256>>> (eager), per launch", nb);
    auto body = [&] {
      for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(chain_k, nb, 256, 0, s, buf, nb);
    };
    for (int i = 0; i < 20; ++i) body();
    hipEventRecord(a, s);
    for (int i = 0; i < R; ++i) body();
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-58s %8.2f us\n", nm, ms * 1e3f / (R * 10));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    body();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ge, s));
    hipEventRecord(a, s);
    for (int i = 0; i < R; ++i) CK(hipGraphLaunch(ge, s));
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    snprintf(nm, sizeof nm, "chain of 10 x chain_k<<<%d,256>>> (hipGraph), per launch", nb);
    printf("%-58s %8.2f us\n", nm, ms * 1e3f / (R * 10));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  // host-side cost of enqueueing (no dependency wait: the GPU runs empty kernels faster than the host
  // submits them, so host time / call is the submission cost)
  {
    auto host_rate = [&](const char *name, auto body) {
      for (int i = 0; i < 200; ++i) body();
      CK(hipStreamSynchronize(s));
      const int R2 = 4000;
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < R2; ++i) body();
      auto t1 = std::chrono::steady_clock::now();
      CK(hipStreamSynchronize(s));
      printf("%-58s %8.2f us/call (host)\n", name, std::chrono::duration<double, std::micro>(t1 - t0).count() / R2);
      // CK's `return 1` makes this lambda return int: without this line the normal path flowed off the end
      // of a non-void function (undefined behaviour; clang -O3 compiles it as unreachable), which is the
      // core dump right after this line's output in profiles/r03/launch_floor.txt (hipcc warned:
      // -Wreturn-type, "non-void lambda does not return a value in all control paths")
      return 0;
    };
    if (host_rate("host: hipLaunchKernelGGL empty<<<1,64>>>", [&] { hipLaunchKernelGGL(empty_k, 1, 64, 0, s); }))
      return 1;
  }
  CK(hipStreamSynchronize(s));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  CK(hipEventDestroy(m));
  CK(hipStreamDestroy(s));
  CK(hipFree(buf));
  CK(hipFree(out));
  CK(hipDeviceSynchronize());
  printf("teardown ok\n");
  return 0;
}
