// Host-side synchronisation of the engine's two concurrency mechanisms, kept free of HIP so that the
// sanitizer harness (tests/host/sanitize_harness.cpp, ThreadSanitizer and AddressSanitizer builds with
// g++) runs them on the CPU:
//   RankBarrier - the reusable generation barrier of the in-process rank group (comm.cpp, LocalComm);
//   TaskFifo    - the S-LBFGS twin's helper thread: tasks run in posting order on one worker thread
//                 (solvers.cpp, SlbfgsSolver), the poster waits for a task by its ticket.
// The reference is single-threaded (src/cuda/common.cuh); neither has a counterpart there.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>

namespace lbf {

// n threads meet; a thread that never arrives (an error on its rank) turns into an error on the others
// after `timeout` instead of a hang, and once broken the barrier stays broken for every later call.
class RankBarrier {
public:
  explicit RankBarrier(int n, std::chrono::milliseconds timeout = std::chrono::seconds(120))
      : n_(n), timeout_(timeout) {}
  // Returns when all n have arrived at this generation. Throws std::runtime_error when the barrier is or
  // becomes broken (break_all from any thread) or the wait times out (which breaks it).
  void arrive_and_wait() {
    std::unique_lock<std::mutex> lk(mu_);
    if (broken_) throw std::runtime_error("local rank group: broken by another rank");
    const unsigned long long g = gen_;
    if (++arrived_ == n_) {
      arrived_ = 0;
      ++gen_;
      cv_.notify_all();
      return;
    }
    // the steady clock (a wall-clock jump cannot stretch or cut the rank-failure timeout); only the
    // ThreadSanitizer build of the host harness waits on a system_clock deadline: libstdc++ maps that to
    // pthread_cond_timedwait, which gcc 11's TSan intercepts, while the steady clock's
    // pthread_cond_clockwait is not intercepted there and reports a bogus double lock
#if defined(__SANITIZE_THREAD__)
    const bool ok = cv_.wait_until(lk, std::chrono::system_clock::now() + timeout_,
                                   [&] { return gen_ != g || broken_; });
#else
    const bool ok = cv_.wait_for(lk, timeout_, [&] { return gen_ != g || broken_; });
#endif
    if (gen_ != g) return;
    broken_ = true;
    lk.unlock();
    cv_.notify_all();
    throw std::runtime_error(ok ? "local rank group: broken by another rank"
                                : "local rank group: a rank did not reach the collective (timeout)");
  }
  void break_all() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      broken_ = true;
    }
    cv_.notify_all();
  }
  bool broken() {
    std::lock_guard<std::mutex> lk(mu_);
    return broken_;
  }
  int size() const { return n_; }

private:
  const int n_;
  const std::chrono::milliseconds timeout_;
  std::mutex mu_;
  std::condition_variable cv_;
  int arrived_ = 0;
  unsigned long long gen_ = 0;
  bool broken_ = false;
};

// One worker thread running posted tasks in order. `init` runs first on the worker (e.g. hipSetDevice);
// if it fails, or a task throws, the FIFO is failed for good: every later task is skipped (its ticket
// still completes) and every later wait() rethrows that first error. The destructor runs (or skips) what is
// queued, then joins.
class TaskFifo {
public:
  explicit TaskFifo(std::function<void()> init = nullptr) {
    th_ = std::thread([this, init]() {
      if (init) {
        try {
          init();
        } catch (...) {
          std::lock_guard<std::mutex> lk(mu_);
          err_ = std::current_exception();
        }
      }
      for (;;) {
        std::function<void()> f;
        bool failed;
        {
          std::unique_lock<std::mutex> lk(mu_);
          cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
          if (q_.empty()) return; // stop requested and nothing left
          f = std::move(q_.front());
          q_.pop_front();
          failed = err_ != nullptr;
        }
        if (!failed) {
          try {
            f();
          } catch (...) {
            std::lock_guard<std::mutex> lk(mu_);
            if (!err_) err_ = std::current_exception();
          }
        }
        done_.fetch_add(1, std::memory_order_release);
      }
    });
  }
  ~TaskFifo() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_one();
    if (th_.joinable()) th_.join();
  }
  TaskFifo(const TaskFifo &) = delete;
  TaskFifo &operator=(const TaskFifo &) = delete;

  // Queues f; returns its ticket (1-based, in posting order). Only the owning thread posts.
  long long post(std::function<void()> f) {
    long long ticket;
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.push_back(std::move(f));
      ticket = ++posted_;
    }
    cv_.notify_one();
    return ticket;
  }
  // Returns once task `ticket` has run (or been skipped); rethrows the first error if the FIFO has failed
  // (sticky: the error is not consumed). ticket <= 0: no-op.
  void wait(long long ticket) {
    if (ticket <= 0) return;
    for (int spin = 0; done_.load(std::memory_order_acquire) < ticket; ++spin)
      if (spin > 64) std::this_thread::yield();
    std::exception_ptr e;
    {
      std::lock_guard<std::mutex> lk(mu_);
      e = err_;
    }
    if (e) std::rethrow_exception(e);
  }
  long long posted() const { return posted_; } // owning thread only
  void wait_all() { wait(posted_); }

private:
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  std::atomic<long long> done_{0};
  long long posted_ = 0;
  std::exception_ptr err_;
  bool stop_ = false;
};

} // namespace lbf
