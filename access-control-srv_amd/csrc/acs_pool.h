// acs_pool.h — the host worker pool of the request codec (acs_codec.cpp).
//
// An encode call runs a dozen parallel phases (delimit, parse + encode, class keys, class rows,
// coherence order, assembly).  Spawning a fresh set of std::threads per phase cost ≈0.4 ms per
// 16-thread phase (measured on the 8-CPU build container), ≈6 ms per call — the pipeline's
// 131,072-request chunks paid it eight times per million requests.  The pool's workers persist
// and wait on a condition variable between phases.
//
// run(n, f): f(t) for t in [0, n), t = 0 on the calling thread.  One run at a time (a second
// caller waits); a run issued from inside a task (a worker, or the caller's own t = 0) runs its
// tasks inline, one after the other, so nested phases cannot deadlock.
#pragma once

#include <condition_variable>
#include <cstdint>
#include <exception>
#include <functional>
#include <mutex>
#include <pthread.h>
#include <thread>
#include <vector>

namespace acs_pool {

class Pool {
 public:
  static Pool& instance() {
    static Pool** p = [] {
      // a forked child has none of the parent's workers: it starts an empty pool
      pthread_atfork(nullptr, nullptr, [] { slot() = new Pool; });
      return &slot();
    }();
    return **p;
  }

  // inline_if_busy: when another run holds the pool, run the tasks inline on this thread instead
  // of waiting for it (batch validation: a pipeline's check of chunk k must not queue behind the
  // encoder phases of chunk k + 1).  An exception thrown by any task is rethrown here, after every
  // worker has finished the run (the first one thrown; the others are dropped).
  void run(int n, const std::function<void(int)>& f, bool inline_if_busy = false) {
    if (n <= 1 || inside()) {
      for (int t = 0; t < n; ++t) f(t);
      return;
    }
    std::unique_lock<std::mutex> one(run_mu_, std::defer_lock);
    if (inline_if_busy) {
      if (!one.try_lock()) {
        for (int t = 0; t < n; ++t) f(t);
        return;
      }
    } else {
      one.lock();
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      grow(n - 1);
      task_ = &f;
      n_ = n;
      pending_ = n - 1;
      error_ = nullptr;
      ++gen_;
    }
    cv_.notify_all();
    std::exception_ptr mine;
    inside() = true;
    try {
      f(0);
    } catch (...) {
      mine = std::current_exception();
    }
    inside() = false;
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return pending_ == 0; });  // no worker still runs f before it unwinds
    task_ = nullptr;
    std::exception_ptr e = mine ? mine : error_;
    error_ = nullptr;
    lk.unlock();
    if (e) std::rethrow_exception(e);
  }

 private:
  static Pool*& slot() {
    static Pool* p = new Pool;  // never destroyed: its workers stay parked until the process ends
    return p;
  }
  static bool& inside() {
    static thread_local bool in = false;
    return in;
  }
  void grow(int m) {  // (mu_ held) workers for task indices 1..m
    while ((int)workers_.size() < m) {
      const int idx = (int)workers_.size();
      const uint64_t g0 = gen_;  // a new worker waits for the next run, not the last one
      workers_.emplace_back([this, idx, g0] { loop(idx, g0); });
      workers_.back().detach();
    }
  }
  void loop(int idx, uint64_t seen) {
    inside() = true;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return gen_ != seen; });
      seen = gen_;
      if (idx + 1 >= n_) continue;
      const std::function<void(int)>* f = task_;
      lk.unlock();
      std::exception_ptr e;
      try {
        (*f)(idx + 1);
      } catch (...) {
        e = std::current_exception();
      }
      lk.lock();
      if (e && !error_) error_ = e;
      if (--pending_ == 0) done_.notify_all();
    }
  }

  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_;
  std::vector<std::thread> workers_;
  const std::function<void(int)>* task_ = nullptr;
  std::exception_ptr error_;  // (mu_) the first exception a worker's task threw this run
  int n_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
};

// f(t) for t in [0, n) on the pool
inline void run(int n, const std::function<void(int)>& f, bool inline_if_busy = false) {
  Pool::instance().run(n, f, inline_if_busy);
}

}  // namespace acs_pool
