// Host-side random streams that must reproduce the reference's libstdc++ draws bit for bit:
// parameter initialisation (src/network.hpp:45-71, src/cuda/network.cuh:36-59) and the synthetic
// MNIST-shaped data recipe of SURVEY.md §8(d). Not on the timed path.
#include "host_rng.hpp"

#include <algorithm>
#include <cmath>
#include <random>

namespace lbf {

void init_params_host(const std::vector<Layer> &layers, unsigned seed, int mode, std::vector<float> &out) {
  size_t n = 0;
  for (auto &L : layers) n += size_t(L.in + 1) * L.out;
  out.assign(n, 0.0f);
  std::mt19937 gen(seed);
  for (auto &L : layers) {
    const size_t w = size_t(L.in) * L.out;
    if (mode == 0) {
      // CPU: normal_distribution<double>(0, scale*sqrt(1/In)) over W and b, fresh per layer.
      const double sd = (L.act == 2 ? 1.41421356 : 1.0) * std::sqrt(1.0 / double(L.in));
      std::normal_distribution<double> dist(0.0, sd);
      for (size_t i = 0; i < w + size_t(L.out); ++i) out[L.off + i] = float(dist(gen));
    } else {
      // CUDA: normal_distribution<float>, weights only, zero biases.
      const float sd = (L.act == 2 ? 1.41421356f : 1.0f) * std::sqrt(1.0f / float(L.in));
      std::normal_distribution<float> dist(0.0f, sd);
      for (size_t i = 0; i < w; ++i) out[L.off + i] = dist(gen);
      for (int i = 0; i < L.out; ++i) out[L.off + w + i] = 0.0f;
    }
  }
}

void synth_mnist_host(long long N, int In, int classes, unsigned seed, float *X, float *Y) {
  std::mt19937 gen(seed);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  std::vector<double> proto(size_t(classes) * In);
  for (auto &v : proto) v = U(gen);
  std::uniform_int_distribution<int> C(0, classes - 1);
  for (long long b = 0; b < N; ++b) {
    const int c = C(gen);
    for (int k = 0; k < classes; ++k) Y[size_t(b) * classes + k] = (k == c) ? 1.0f : 0.0f;
    for (int i = 0; i < In; ++i) {
      double v = 0.5 * proto[size_t(c) * In + i] + 0.5 * U(gen);
      v = std::min(1.0, std::max(0.0, v));
      X[size_t(b) * In + i] = float(std::round(255.0 * v) / 255.0);
    }
  }
}

} // namespace lbf
