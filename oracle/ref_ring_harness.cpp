// oracle/ref_ring_harness.cpp — TEST INFRASTRUCTURE ONLY.
// Drives the reference's OWN RingBuffer (src/minimizer/ring_buffer.hpp, the only Eigen-free file on the
// hot path) straight from /root/reference via -I; nothing of it is copied into this repo.
// Output format matches oracle_ring_trace(): one line per push, "head c0 c1 ... c{cap-1}" (-1 = empty).
#include "ring_buffer.hpp"
#include <cstdio>
#include <cstdlib>

int main(int argc, char **argv) {
  const int cap = argc > 1 ? std::atoi(argv[1]) : 3;
  const int npush = argc > 2 ? std::atoi(argv[2]) : 8;
  cpu_mlp::RingBuffer<int> r(static_cast<size_t>(cap));
  for (int t = 0; t < npush; ++t) {
    r.push_back(t);
    // head is private in the reference; recover it as the physical slot of logical index 0,
    // i.e. the position of the oldest element, which is t+1-size modulo cap.
    int head = static_cast<int>((t + 1 - static_cast<int>(r.size())) % cap);
    std::printf("%d", head);
    for (int i = 0; i < cap; ++i) std::printf(" %d", i < static_cast<int>(r.size()) ? r[static_cast<size_t>(i)] : -1);
    std::printf("\n");
  }
  return 0;
}
