#pragma once

#include "runtime.hpp"

#include <vector>

namespace lbf {

// mode 0: CPU stream (all params, double draws), 1: CUDA stream (weights, float draws, zero bias).
void init_params_host(const std::vector<Layer> &layers, unsigned seed, int mode, std::vector<float> &out);
void synth_mnist_host(long long N, int In, int classes, unsigned seed, float *X, float *Y);

} // namespace lbf
