// Internal runtime support for liblbfgs_amd_abi3.so: error type, HIP checks, RAII device buffers.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

namespace lbf {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

#define LBF_HIP(expr)                                                                                        \
  do {                                                                                                       \
    hipError_t e_ = (expr);                                                                                  \
    if (e_ != hipSuccess)                                                                                    \
      throw ::lbf::Error(2, std::string("HIP error: ") + #expr + " -> " + hipGetErrorString(e_) + " (" +     \
                                __FILE__ + ":" + std::to_string(__LINE__) + ")");                            \
  } while (0)

#define LBF_KERNEL_CHECK() LBF_HIP(hipGetLastError())

#define LBF_REQUIRE(cond, msg)                                                                               \
  do {                                                                                                       \
    if (!(cond)) throw ::lbf::Error(1, std::string("invalid argument: ") + (msg));                           \
  } while (0)

// RAII device allocation (the reference's DeviceBuffer, src/cuda/device_buffer.cuh:7-96, minus the
// synchronous copies: everything here is stream-ordered).
template <class T> class DevBuf {
public:
  DevBuf() = default;
  explicit DevBuf(size_t n) { resize(n); }
  ~DevBuf() { release(); }
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
  DevBuf(DevBuf &&o) noexcept : p_(o.p_), n_(o.n_) { o.p_ = nullptr; o.n_ = 0; }
  DevBuf &operator=(DevBuf &&o) noexcept {
    if (this != &o) { release(); p_ = o.p_; n_ = o.n_; o.p_ = nullptr; o.n_ = 0; }
    return *this;
  }
  void resize(size_t n) {
    if (n == n_) return;
    release();
    if (n) LBF_HIP(hipMalloc(&p_, n * sizeof(T)));
    n_ = n;
  }
  void ensure(size_t n) { if (n > n_) resize(n); }
  T *get() const { return p_; }
  size_t size() const { return n_; }
  void release() {
    if (p_) (void)hipFree(p_);
    p_ = nullptr;
    n_ = 0;
  }

private:
  T *p_ = nullptr;
  size_t n_ = 0;
};

// Pinned host staging (status read-back, index uploads).
template <class T> class PinnedBuf {
public:
  PinnedBuf() = default;
  ~PinnedBuf() { if (p_) (void)hipHostFree(p_); }
  PinnedBuf(const PinnedBuf &) = delete;
  PinnedBuf &operator=(const PinnedBuf &) = delete;
  void ensure(size_t n) {
    if (n <= n_) return;
    if (p_) (void)hipHostFree(p_);
    LBF_HIP(hipHostMalloc(&p_, n * sizeof(T), hipHostMallocDefault));
    n_ = n;
  }
  T *get() const { return p_; }
  T &operator[](size_t i) { return p_[i]; }

private:
  T *p_ = nullptr;
  size_t n_ = 0;
};

inline long long cdiv(long long a, long long b) { return (a + b - 1) / b; }
// Integer tuning knob from the environment (read once by the caller's static).
inline int env_int(const char *name, int dflt) {
  const char *e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}

// Extra flags for the library's events: every event orders work on ONE device (profiling marks, the
// S-LBFGS twin's fork / join), so a device-scope release is enough. The default system-scope release writes
// back and invalidates the caches at each record, which costs the recording stream time and leaves the next
// kernel with a cold L2.
inline unsigned event_release_flags() { return unsigned(hipEventReleaseToDevice); }

// Phase timestamps for kernel tuning (debug build only: make ktrace). KT(slot) stores the 100 MHz
// wall clock from thread 0 of block (0,0,0); lbf_dbg_ktrace() copies the slots to the host.
#ifdef LBF_KTRACE
static __device__ unsigned long long lbf_kt_buf[256]; // one per translation unit (no RDC)
#define KT(slot)                                                                                        \
  do {                                                                                                  \
    if ((blockIdx.x | blockIdx.y | blockIdx.z | threadIdx.x) == 0) lbf_kt_buf[slot] = wall_clock64();                         \
  } while (0)
#define KTC(slot)                                                                                       \
  do {                                                                                                  \
    if ((blockIdx.x | blockIdx.y | blockIdx.z | threadIdx.x) == 0) lbf_kt_buf[slot] = clock64();                              \
  } while (0)
// KTF(slot): thread 0 of whichever block runs it (one-block phases: the tail's fin, hist_core)
#define KTF(slot)                                                                                       \
  do {                                                                                                  \
    if (threadIdx.x == 0) lbf_kt_buf[slot] = wall_clock64();                                            \
  } while (0)
// KTB(slot): per-block stamps (thread 0 of every block with blockIdx.z == 0, first 1024 blocks) for
// the distribution of phase times across the grid.
static __device__ unsigned long long lbf_kt_blk[8 * 1024];
#define KTB(slot)                                                                                       \
  do {                                                                                                  \
    const unsigned lin_ = blockIdx.y * gridDim.x + blockIdx.x;                                          \
    if (threadIdx.x == 0 && blockIdx.z == 0 && lin_ < 1024) lbf_kt_blk[(slot) * 1024 + lin_] = wall_clock64(); \
  } while (0)
// KTHW(): where the block runs (XCC id << 32 | HW_ID: CU, shader array, SE, SIMD), for the per-block stamps
static __device__ unsigned long long lbf_kt_hw[1024];
#define KTHW()                                                                                          \
  do {                                                                                                  \
    const unsigned lin_ = blockIdx.y * gridDim.x + blockIdx.x;                                          \
    if (threadIdx.x == 0 && blockIdx.z == 0 && lin_ < 1024) {                                           \
      unsigned xcc_, hw_;                                                                               \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));                                \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));                                  \
      lbf_kt_hw[lin_] = ((unsigned long long)xcc_ << 32) | hw_;                                         \
    }                                                                                                   \
  } while (0)
#else
#define KTHW()                                                                                          \
  do {                                                                                                  \
  } while (0)
#define KTF(slot)                                                                                       \
  do {                                                                                                  \
  } while (0)
#define KTB(slot)                                                                                       \
  do {                                                                                                  \
  } while (0)
#define KTC(slot)                                                                                       \
  do {                                                                                                  \
  } while (0)
#define KT(slot)                                                                                        \
  do {                                                                                                  \
  } while (0)
#endif

} // namespace lbf
