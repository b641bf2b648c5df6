// Activation functions (src/layer.hpp:16-47 forward; derivatives through the post-activation value y,
// src/cuda/kernels.cuh:109-133, equal to the CPU path's act'(Z) in exact arithmetic).
//
// act_c / dact_c take the activation as a template constant; with_act() switches ONCE on the
// (wave-uniform) runtime code and runs a body instantiated per activation, so element loops carry no
// per-element branch tree (a scalar branch per element costs an instruction-fetch redirect each,
// which dominated the GEMM epilogues when the switch sat inside them).
#pragma once

#include "kernels.hpp"

#include <hip/hip_runtime.h>

#include <type_traits>

namespace lbf {

template <int A> __device__ __forceinline__ float act_c(float x) {
  if constexpr (A == ACT_TANH) return tanhf(x);
  else if constexpr (A == ACT_RELU) return x > 0.0f ? x : 0.0f;
  else if constexpr (A == ACT_SIGMOID) return 1.0f / (1.0f + expf(-x));
  else return x;
}
template <int A> __device__ __forceinline__ float dact_c(float y) {
  if constexpr (A == ACT_TANH) return 1.0f - y * y;
  else if constexpr (A == ACT_RELU) return y > 0.0f ? 1.0f : 0.0f;
  else if constexpr (A == ACT_SIGMOID) return y * (1.0f - y);
  else return 1.0f;
}

template <class F> __device__ __forceinline__ void with_act(int a, F &&f) {
  switch (a) {
  case ACT_TANH: f(std::integral_constant<int, ACT_TANH>{}); break;
  case ACT_RELU: f(std::integral_constant<int, ACT_RELU>{}); break;
  case ACT_SIGMOID: f(std::integral_constant<int, ACT_SIGMOID>{}); break;
  default: f(std::integral_constant<int, ACT_LINEAR>{}); break;
  }
}

// Runtime-coded forms for scalar (non-loop) uses.
__device__ __forceinline__ float act_rt(int a, float x) {
  switch (a) {
  case ACT_TANH: return act_c<ACT_TANH>(x);
  case ACT_RELU: return act_c<ACT_RELU>(x);
  case ACT_SIGMOID: return act_c<ACT_SIGMOID>(x);
  default: return x;
  }
}
__device__ __forceinline__ float dact_rt(int a, float y) {
  switch (a) {
  case ACT_TANH: return dact_c<ACT_TANH>(y);
  case ACT_RELU: return dact_c<ACT_RELU>(y);
  case ACT_SIGMOID: return dact_c<ACT_SIGMOID>(y);
  default: return 1.0f;
  }
}

} // namespace lbf
