// Exact Hessian-vector product of the MLP's MSE loss (Pearlmutter's R-operator), SURVEY.md §8(f)
// rank 4: the option that replaces S-LBFGS's finite-difference HVP (s_lbfgs.hpp:88-101, which loses
// ~1e-2 relative to fp32 cancellation) by H(w) v computed in one forward + backward R-pass.
//
// With Z_l = A_{l-1} W_l + b_l, A_l = act_l(Z_l), e = (A_L - y) * s (s = inv_scale),
// dZ_L = e .* act'_L, delta_{l-1} = dZ_l W_l^T, dZ_{l-1} = delta_{l-1} .* act'_{l-1}, and the
// direction V = [V_l ; v_l] in the parameter layout:
//   R{Z_l}  = R{A_{l-1}} W_l + A_{l-1} V_l + v_l          (R{A_{-1}} = R{X} = 0)
//   R{A_l}  = act'_l .* R{Z_l}
//   R{dZ_L} = s (act'_L^2 + (A_L - y) act''_L) .* R{Z_L}
//   R{dZ_{l-1}} = (R{dZ_l} W_l^T + dZ_l V_l^T) .* act'_{l-1} + delta_{l-1} .* act''_{l-1} .* R{Z_{l-1}}
//   (H v)_l = [A_{l-1} | 1]^T R{dZ_l} + [R{A_{l-1}} | 0]^T dZ_l   (+ lambda v)
// The products are the engine's MFMA GEMMs (runtime.cpp Mlp::hvp); this file holds the elementwise
// R-steps. act' and act'' are taken through the post-activation value a (act.hpp convention):
// tanh 1-a^2, -2a(1-a^2); sigmoid a(1-a), a(1-a)(1-2a); relu [a>0], 0; linear 1, 0.
#include "act.hpp"
#include "internal.hpp"
#include "kernels.hpp"

#include <hip/hip_runtime.h>

namespace lbf {

namespace {

__device__ __forceinline__ float d2act_rt(int act, float a) {
  switch (act) {
  case ACT_TANH: return -2.0f * a * (1.0f - a * a);
  case ACT_SIGMOID: return a * (1.0f - a) * (1.0f - 2.0f * a);
  default: return 0.0f;
  }
}

// RA = act'(A) .* RZ
__global__ __launch_bounds__(256) void rop_act_kernel(long long n, const float *A, const float *RZ, int act,
                                                      float *RA) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) RA[e] = dact_rt(act, A[e]) * RZ[e];
}

// RdZ = s (act'(A)^2 + (A - y) act''(A)) .* RZ on the output layer (rows gathered by idx)
__global__ __launch_bounds__(256) void rop_out_kernel(long long B, int Out, const float *A, const float *Y,
                                                      const int *idx, const float *RZ, int act, float s,
                                                      float *RdZ) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * Out) return;
  const long long b = e / Out;
  const int o = int(e - b * Out);
  const float a = A[e], y = Y[(idx ? (long long)idx[b] : b) * Out + o];
  const float d1 = dact_rt(act, a);
  RdZ[e] = s * (d1 * d1 + (a - y) * d2act_rt(act, a)) * RZ[e];
}

// out = T1 + T2 (+ delta .* act''(A) .* RZ when delta is non-null)
__global__ __launch_bounds__(256) void rop_back_kernel(long long n, const float *T1, const float *T2, const float *delta,
                                                       const float *A, const float *RZ, int act, float *out) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  float v = T1[e] + T2[e];
  if (delta) v += delta[e] * d2act_rt(act, A[e]) * RZ[e];
  out[e] = v;
}

} // namespace

void rop_act(hipStream_t s, long long n, const float *A, const float *RZ, int act, float *RA) {
  if (n <= 0) return;
  hipLaunchKernelGGL(rop_act_kernel, dim3(unsigned(cdiv(n, 256))), dim3(256), 0, s, n, A, RZ, act, RA);
  LBF_KERNEL_CHECK();
}

void rop_out(hipStream_t s, long long B, int Out, const float *A, const float *Y, const int *idx, const float *RZ,
             int act, double inv_scale, float *RdZ) {
  if (B <= 0) return;
  hipLaunchKernelGGL(rop_out_kernel, dim3(unsigned(cdiv(B * Out, 256))), dim3(256), 0, s, B, Out, A, Y, idx, RZ, act,
                     float(inv_scale), RdZ);
  LBF_KERNEL_CHECK();
}

void rop_back(hipStream_t s, long long n, const float *T1, const float *T2, const float *delta, const float *A,
              const float *RZ, int act, float *out) {
  if (n <= 0) return;
  hipLaunchKernelGGL(rop_back_kernel, dim3(unsigned(cdiv(n, 256))), dim3(256), 0, s, n, T1, T2, delta, A, RZ, act,
                     out);
  LBF_KERNEL_CHECK();
}

bool act_has_d2(int act) { return act == ACT_TANH || act == ACT_SIGMOID; }

} // namespace lbf
