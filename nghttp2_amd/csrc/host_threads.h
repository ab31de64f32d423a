// host_threads.h -- the host worker threads of the batched front-ends.
//
// The inflate/deflate front-ends (hd_inflate.cpp, hd_deflate.cpp) do their
// table work per connection, and connections are independent, so a batch of
// many connections spreads over host threads: one task per connection, or per
// block for the stateless parse.  The workers are started once per process
// and parked between calls; a call hands them a job and works on it itself.
// NGHTTP2_AMD_HOST_THREADS sets the count; the default is the hardware
// threads, capped at 16 (the host share of one GPU on the MI355X boxes).
// NGHTTP2_AMD_TRACE=1 prints each call's phase times to stderr.
#pragma once

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

namespace nghttp2_amd_host {

inline unsigned host_threads() {
  static const unsigned t = [] {
    long n = (long)std::thread::hardware_concurrency();
    if (const char *e = getenv("NGHTTP2_AMD_HOST_THREADS")) n = atol(e);
    else n = std::min(n, 16L);
    return (unsigned)std::max(1L, std::min(n, 256L));
  }();
  return t;
}

// A spin-wait hint for the busy loops below (x86 `pause`; a no-op elsewhere).
inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#endif
}

class Pool {
 public:
  static Pool &get() {
    static Pool *p = new Pool(host_threads() - 1);  // never destroyed: workers park until exit
    return *p;
  }
  unsigned workers() const { return (unsigned)th_.size(); }
  // Runs fn on every worker and on the caller; returns when all are done.
  // Calls from several host threads take turns.
  void run(const std::function<void()> &fn) {
    std::lock_guard<std::mutex> turn(run_mu_);
    job_.v.store(&fn, std::memory_order_relaxed);
    active_.v.store((unsigned)th_.size(), std::memory_order_relaxed);
    bool wake;
    {
      std::lock_guard<std::mutex> l(mu_);
      gen_.v.fetch_add(1, std::memory_order_release);
      wake = sleepers_ > 0;
    }
    if (wake) cv_.notify_all();
    fn();
    for (unsigned i = 0; active_.v.load(std::memory_order_acquire) != 0; ++i) {
      if (i < 4096) cpu_relax();
      else std::this_thread::yield();
    }
    job_.v.store(nullptr, std::memory_order_relaxed);
  }
  // A front-end call that runs several parallel phases holds a CallScope for
  // its whole duration: while one is open, a worker that finishes a phase
  // spins (with a pause) for the next one, up to spin_us(), instead of
  // parking on the condition variable, so the call's phases hand over without
  // a futex wake-up each.  With no call open the workers park at once, so an
  // embedding application's threads never compete with idle spinning
  // (round 6; round 5 spun 200 us after every phase, call or not).
  class CallScope {
   public:
    CallScope() { calls().v.fetch_add(1, std::memory_order_relaxed); }
    ~CallScope() { calls().v.fetch_sub(1, std::memory_order_relaxed); }
    CallScope(const CallScope &) = delete;
    CallScope &operator=(const CallScope &) = delete;
  };

 private:
  // NGHTTP2_AMD_SPIN_US (default 200; 0: always park at once): the longest a
  // worker spins between the phases of an open call
  static int spin_us() {
    static const int v = [] {
      const char *e = getenv("NGHTTP2_AMD_SPIN_US");
      return e ? std::max(0, atoi(e)) : 200;
    }();
    return v;
  }
  explicit Pool(unsigned n) {
    for (unsigned k = 0; k < n; ++k) {
      try {
        th_.emplace_back([this] { loop(); });
        th_.back().detach();
      } catch (const std::system_error &) {
        break;
      }
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      // spin for the next job while a call is open (at most spin_us()), then park
      bool got = false;
      const auto t0 = std::chrono::steady_clock::now();
      for (unsigned i = 0;; ++i) {
        if (gen_.v.load(std::memory_order_acquire) != seen) {
          got = true;
          break;
        }
        if (calls().v.load(std::memory_order_relaxed) == 0) break;
        if ((i & 255u) == 255u &&
            std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us()))
          break;
        cpu_relax();
      }
      if (!got) {
        std::unique_lock<std::mutex> l(mu_);
        ++sleepers_;
        cv_.wait(l, [&] { return gen_.v.load(std::memory_order_relaxed) != seen; });
        --sleepers_;
      }
      seen = gen_.v.load(std::memory_order_acquire);
      (*job_.v.load(std::memory_order_relaxed))();
      active_.v.fetch_sub(1, std::memory_order_acq_rel);
    }
  }
  // (each shared word on its own cache line: the workers' decrements of
  // active_ must not bounce the line the spinning workers poll gen_ on)
  template <class T>
  struct alignas(64) Line {
    std::atomic<T> v{};
  };
  std::vector<std::thread> th_;
  std::mutex run_mu_, mu_;
  std::condition_variable cv_;
  Line<const std::function<void()> *> job_;
  Line<unsigned> active_;
  Line<uint64_t> gen_;
  static Line<int> &calls() {  // open CallScopes (no pool is started for one)
    static Line<int> c;
    return c;
  }
  unsigned sleepers_ = 0;  // (under mu_)
};

// f(i) for i in [0, n), `grain` consecutive indices per fetch; serial when
// there are fewer than two grains of work.
template <class F>
void parallel_for(size_t n, size_t grain, F &&f) {
  if (grain == 0) grain = 1;
  if (n < 2 * grain || host_threads() <= 1) {
    for (size_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::atomic<size_t> next{0};
  const std::function<void()> work = [&]() {
    for (;;) {
      const size_t a = next.fetch_add(grain, std::memory_order_relaxed);
      if (a >= n) return;
      const size_t b = std::min(n, a + grain);
      for (size_t i = a; i < b; ++i) f(i);
    }
  };
  Pool::get().run(work);
}

inline bool trace_on() {
  static const bool on = getenv("NGHTTP2_AMD_TRACE") != nullptr;
  return on;
}

// Phase times of one call, printed at the end of the call when tracing.
class Phases {
 public:
  explicit Phases(const char *who) : who_(who), on_(trace_on()), t_(std::chrono::steady_clock::now()) {}
  void mark(const char *name) {
    if (!on_) return;
    const auto now = std::chrono::steady_clock::now();
    char b[96];
    snprintf(b, sizeof b, " %s=%.1fus", name, std::chrono::duration<double, std::micro>(now - t_).count());
    log_ += b;
    t_ = now;
  }
  ~Phases() {
    if (on_) fprintf(stderr, "[nghttp2_amd %s]%s\n", who_, log_.c_str());
  }

 private:
  const char *who_;
  bool on_;
  std::chrono::steady_clock::time_point t_;
  std::string log_;
};

}  // namespace nghttp2_amd_host
