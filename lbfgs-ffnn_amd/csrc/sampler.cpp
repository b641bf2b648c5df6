// Minibatch index sampling (see sampler.hpp): SLBFGS::sample_minibatch_indices (s_lbfgs.hpp:141-160).
#include "sampler.hpp"

#include <numeric>
#include <utility>

namespace lbf {

MinibatchSampler::MinibatchSampler(size_t N) : perm_(N) { std::iota(perm_.begin(), perm_.end(), size_t(0)); }

size_t MinibatchSampler::draw(size_t b, std::mt19937 &rng, std::vector<int> &out) {
  // s_lbfgs.hpp:141-160: partial Fisher-Yates over iota(N), uniform_int_distribution<size_t>(i, N-1).
  const size_t N = perm_.size();
  if (N == 0 || b == 0) return 0;
  if (b >= N) { // the whole identity, no draws
    for (size_t i = 0; i < N; ++i) out.push_back(int(i));
    return N;
  }
  touched_.resize(b);
  for (size_t i = 0; i < b; ++i) {
    std::uniform_int_distribution<size_t> dist(i, N - 1);
    const size_t j = dist(rng);
    touched_[i] = j;
    std::swap(perm_[i], perm_[j]);
  }
  for (size_t i = 0; i < b; ++i) out.push_back(int(perm_[i]));
  for (size_t i = b; i-- > 0;) std::swap(perm_[i], perm_[touched_[i]]); // undo in reverse: identity again
  return b;
}

std::vector<size_t> sample_minibatch(size_t N, size_t b, std::mt19937 &rng) {
  MinibatchSampler smp(N);
  std::vector<int> v;
  smp.draw(b, rng, v);
  return std::vector<size_t>(v.begin(), v.end());
}

} // namespace lbf
