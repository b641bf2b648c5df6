// Host-only sanitizer harness: the engine's two concurrency mechanisms and the minibatch
// sampler, driven on the CPU with stub "launches" in place of HIP calls. Built twice by
// tests/test_host_sanitizers.py, with -fsanitize=thread and with -fsanitize=address,undefined:
//   1. RankBarrier (host_sync.hpp) under the in-process rank group's protocol (comm.cpp LocalComm): every
//      rank publishes its buffer pointer and count, meets, reads every other rank's, meets again; a rank
//      that throws breaks the group and the others fail instead of hanging.
//   2. TaskFifo (host_sync.hpp) under the S-LBFGS twin's protocol (solvers.cpp epoch_steps): tasks posted in
//      order, the poster waits by ticket before reading what a task produced, an error fails the FIFO for good
//      (every later task skipped, every later wait rethrows), the destructor runs what is queued.
//   3. MinibatchSampler (sampler.cpp) against a plain restatement of s_lbfgs.hpp:141-160 (iota(N) per draw).
#include "host_sync.hpp"
#include "sampler.hpp"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

using namespace lbf;

#define CHECK(c)                                                                                         \
  do {                                                                                                   \
    if (!(c)) {                                                                                          \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);                          \
      std::exit(1);                                                                                      \
    }                                                                                                    \
  } while (0)

// ---- 1. rank group ---------------------------------------------------------------------------------
struct Group { // LocalGroup's host state (comm.cpp), the device buffers replaced by host vectors
  explicit Group(int n, int timeout_ms) : bar(n, std::chrono::milliseconds(timeout_ms)), bufs(n), counts(n) {}
  RankBarrier bar;
  std::vector<const float *> bufs;
  std::vector<size_t> counts;
};

// One collective of rank r: publish, meet, sum everyone's buffer in rank order, meet again (nobody
// overwrites a buffer before every rank has read it), then the result into this rank's buffer.
static void allreduce(Group &G, int r, std::vector<float> &buf) {
  G.bufs[size_t(r)] = buf.data();
  G.counts[size_t(r)] = buf.size();
  G.bar.arrive_and_wait();
  std::vector<float> sum(buf.size(), 0.0f);
  for (int j = 0; j < G.bar.size(); ++j) {
    CHECK(G.counts[size_t(j)] == buf.size());
    for (size_t i = 0; i < buf.size(); ++i) sum[i] += G.bufs[size_t(j)][i];
  }
  G.bar.arrive_and_wait();
  buf = sum;
}

static void test_rank_group() {
  for (int n : {2, 3, 4, 8}) {
    Group G(n, 20000);
    std::vector<std::thread> th;
    std::atomic<int> bad{0};
    for (int r = 0; r < n; ++r)
      th.emplace_back([&, r]() {
        for (int it = 0; it < 200; ++it) {
          std::vector<float> b(64 + (it % 5), float(r + 1) * float(it + 1));
          allreduce(G, r, b);
          const float want = float(n * (n + 1) / 2) * float(it + 1);
          for (float v : b)
            if (v != want) bad.fetch_add(1);
        }
      });
    for (auto &t : th) t.join();
    CHECK(bad.load() == 0);
  }
  // a rank that fails (throws before the collective) must turn into errors on the others, not a hang
  {
    const int n = 4;
    Group G(n, 300);
    std::atomic<int> errs{0};
    std::vector<std::thread> th;
    for (int r = 0; r < n; ++r)
      th.emplace_back([&, r]() {
        try {
          std::vector<float> b(16, 1.0f);
          allreduce(G, r, b);
          if (r == 2) throw std::runtime_error("rank 2 fails");
          allreduce(G, r, b);
        } catch (const std::runtime_error &) {
          errs.fetch_add(1);
          G.bar.break_all();
        }
      });
    for (auto &t : th) t.join();
    CHECK(errs.load() == n);
    CHECK(G.bar.broken());
  }
}

// ---- 2. twin worker ----------------------------------------------------------------------------------
static void test_task_fifo() {
  // in-order execution; the poster reads a task's output only after waiting for its ticket (solvers.cpp:
  // twin_wait(tk[t]) before the context stream waits on the event task t records)
  {
    std::atomic<bool> init_ran{false};
    TaskFifo q([&]() { init_ran.store(true); });
    const int T = 2000;
    std::vector<long long> out(T, -1); // written by the worker, read by the poster after wait()
    std::vector<long long> tk(T, 0);
    long long order = 0;               // touched by the worker only
    for (int t = 0; t < T; ++t) {
      tk[size_t(t)] = q.post([&out, &order, t]() { out[size_t(t)] = order++; });
      if (t >= 2) { // the epoch's pattern: step t waits for task t - 2 (two steps ahead)
        q.wait(tk[size_t(t - 2)]);
        CHECK(out[size_t(t - 2)] == t - 2);
      }
    }
    q.wait_all();
    for (int t = 0; t < T; ++t) CHECK(out[size_t(t)] == t);
    CHECK(init_ran.load());
  }
  // an error fails the FIFO for good: later tasks are skipped, every later wait rethrows it
  {
    TaskFifo q;
    std::vector<int> ran(6, 0);
    q.post([&]() { ran[0] = 1; });
    const long long bad = q.post([&]() {
      ran[1] = 1;
      throw std::runtime_error("launch failed");
    });
    const long long skipped = q.post([&]() { ran[2] = 1; });
    int thrown = 0;
    try {
      q.wait(skipped);
    } catch (const std::runtime_error &) {
      ++thrown;
    }
    CHECK(thrown == 1 && bad == 2);
    const long long after = q.post([&]() { ran[3] = 1; });
    try {
      q.wait(after); // still failed: the error is sticky, the task skipped
    } catch (const std::runtime_error &) {
      ++thrown;
    }
    CHECK(thrown == 2);
    CHECK(ran[0] == 1 && ran[1] == 1 && ran[2] == 0 && ran[3] == 0);
  }
  // a failing init (hipSetDevice on the worker) skips every task, the first wait reports it and so does
  // every later one (a task must never run on a thread whose device was not set)
  {
    TaskFifo q([]() { throw std::runtime_error("no device"); });
    int ran = 0;
    int thrown = 0;
    for (int k = 0; k < 3; ++k) {
      const long long t = q.post([&]() { ran = 1; });
      try {
        q.wait(t);
      } catch (const std::runtime_error &) {
        ++thrown;
      }
    }
    CHECK(thrown == 3 && ran == 0);
  }
  // the destructor runs what is still queued, then joins (the solver's teardown)
  {
    std::atomic<int> n{0};
    {
      TaskFifo q;
      for (int i = 0; i < 500; ++i) q.post([&]() { n.fetch_add(1); });
    }
    CHECK(n.load() == 500);
  }
}

// ---- 3. sampler --------------------------------------------------------------------------------------
static std::vector<int> reference_draw(size_t N, size_t b, std::mt19937 &rng) { // s_lbfgs.hpp:141-160
  std::vector<size_t> idx(N);
  std::iota(idx.begin(), idx.end(), size_t(0));
  const size_t bb = std::min(b, N);
  for (size_t i = 0; i < bb && b < N; ++i) {
    std::uniform_int_distribution<size_t> dist(i, N - 1);
    std::swap(idx[i], idx[dist(rng)]);
  }
  return std::vector<int>(idx.begin(), idx.begin() + long(bb));
}

static void test_sampler() {
  for (size_t N : {1u, 7u, 100u, 1000u, 60000u})
    for (size_t b : {1u, 2u, 32u, 256u, 1000u, 70000u}) {
      std::mt19937 r1(123), r2(123);
      MinibatchSampler smp(N);
      for (int call = 0; call < 20; ++call) {
        std::vector<int> got;
        const size_t k = smp.draw(b, r1, got);
        const std::vector<int> want = reference_draw(N, b, r2);
        CHECK(k == want.size() && got == want);
      }
    }
}

// A deliberate unsynchronised write/write pair: the pytest runs it once to prove the sanitizer build is live
// (ThreadSanitizer must report it).
static void canary_race() {
  static int shared = 0;
  std::thread a([]() { for (int i = 0; i < 1000; ++i) shared = shared + 1; });
  std::thread b([]() { for (int i = 0; i < 1000; ++i) shared = shared + 2; });
  a.join();
  b.join();
  std::printf("canary %d\n", shared);
}

int main(int argc, char **argv) {
  if (argc > 1 && std::string(argv[1]) == "canary") {
    canary_race();
    return 0;
  }
  test_rank_group();
  test_task_fifo();
  test_sampler();
  std::printf("sanitize harness ok\n");
  return 0;
}
