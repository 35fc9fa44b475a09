// pool.hpp — a small persistent worker pool for the host encoder's per-pod
// passes.  parallel_for(n, grain, fn) runs fn(begin, end) over chunks of
// [0, n) on up to SR_HOST_THREADS (default min(16, hardware)) threads and
// returns when every chunk is done.  Results must not depend on the thread
// count: callers write disjoint slots and merge serially.
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace sr {

class Pool {
 public:
  static Pool& get() {
    static Pool pool;
    return pool;
  }

  size_t threads() const { return workers_.size() + 1; }

  void parallel_for(size_t n, size_t grain, const std::function<void(size_t, size_t)>& fn) {
    if (n == 0) return;
    if (workers_.empty() || n <= grain) {
      fn(0, n);
      return;
    }
    std::unique_lock<std::mutex> lk(mu_);
    job_ = &fn;
    n_ = n;
    grain_ = grain;
    next_.store(0);
    gen_.fetch_add(1, std::memory_order_release);
    cv_.notify_all();
    lk.unlock();
    run_chunks();
    // every chunk is claimed; the workers that claimed one are counted in
    // in_flight_ (they joined under the lock before claiming)
    lk.lock();
    done_cv_.wait(lk, [&] { return in_flight_ == 0; });
    job_ = nullptr;  // a worker waking for this generation now skips it
  }

  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  Pool() {
    unsigned hw = std::thread::hardware_concurrency();
    unsigned want = std::min(16u, hw ? hw : 1u);
    if (const char* e = std::getenv("SR_HOST_THREADS")) want = static_cast<unsigned>(std::max(1, std::atoi(e)));
    if (const char* e = std::getenv("SR_HOST_SPIN")) spin_ = std::max(0, std::atoi(e));
    for (unsigned i = 1; i < want; ++i) workers_.emplace_back([this] { loop(); });
  }

  void run_chunks() {
    for (;;) {
      const size_t b = next_.fetch_add(grain_);
      if (b >= n_) return;
      (*job_)(b, std::min(n_, b + grain_));
    }
  }

  // A worker spins a little (~tens of microseconds) for the next generation
  // before it sleeps: a host phase issues parallel loops back to back, and a
  // condition-variable wake-up per loop and worker costs more than the loop.
  // SR_HOST_SPIN sets the spin count (0: sleep at once, for a planner sharing
  // its cores with other work).
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      for (int i = 0; i < spin_ && gen_.load(std::memory_order_acquire) == seen; ++i) {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#elif defined(__aarch64__)
        asm volatile("yield");
#else
        if ((i & 63) == 63) std::this_thread::yield();
#endif
      }
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return gen_.load(std::memory_order_relaxed) != seen; });
      seen = gen_.load(std::memory_order_relaxed);
      if (stop_) return;
      if (!job_) continue;  // that generation's loop is over
      ++in_flight_;
      lk.unlock();
      run_chunks();
      lk.lock();
      if (--in_flight_ == 0) done_cv_.notify_one();
    }
  }

  int spin_ = 4000;
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(size_t, size_t)>* job_ = nullptr;
  size_t n_ = 0, grain_ = 1;
  std::atomic<size_t> next_{0};
  size_t in_flight_ = 0;
  std::atomic<uint64_t> gen_{0};
  bool stop_ = false;
};

inline size_t pool_threads() { return Pool::get().threads(); }

inline void parallel_for(size_t n, size_t grain, const std::function<void(size_t, size_t)>& fn) {
  Pool::get().parallel_for(n, grain, fn);
}

}  // namespace sr
