// Minibatch index sampling of S-LBFGS (host only, no HIP: the sanitizer harness links it with g++).
#pragma once

#include <cstddef>
#include <random>
#include <vector>

namespace lbf {

// libstdc++ partial Fisher-Yates (s_lbfgs.hpp:141-160) over a reusable identity permutation of N: a draw
// swaps b positions, reads them, and swaps them back (O(b) per minibatch instead of the reference's iota(N),
// which cost ~15 ms of host time per cfg-4 epoch); the draws and results are the reference's.
class MinibatchSampler {
 public:
  explicit MinibatchSampler(size_t N);
  // appends the minibatch (min(b, N) indices) to out; returns how many
  size_t draw(size_t b, std::mt19937 &rng, std::vector<int> &out);

 private:
  std::vector<size_t> perm_, touched_;
};
// One draw with a fresh sampler (the ABI helper).
std::vector<size_t> sample_minibatch(size_t N, size_t b, std::mt19937 &rng);

} // namespace lbf
