#pragma once

#include "runtime.hpp"

#include <vector>

namespace lbf {

// mode 0: CPU stream (all params, double draws), 1: CUDA stream (weights, float draws, zero bias).
void init_params_host(const std::vector<Layer> &layers, unsigned seed, int mode, std::vector<float> &out);
void synth_mnist_host(long long N, int In, int classes, unsigned seed, float *X, float *Y);

// IDX files (idx.cpp; the reference's tests/mnist/mnist_loader.hpp). h_out == nullptr: header only.
void idx_read_images(const char *path, long long max_images, float *h_out, long long *count, int *rows, int *cols);
void idx_read_labels(const char *path, long long max_labels, int classes, float *h_onehot, long long *count);

} // namespace lbf
