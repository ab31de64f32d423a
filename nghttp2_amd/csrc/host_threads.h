// host_threads.h -- the host worker threads of the batched front-ends.
//
// The inflate/deflate front-ends (hd_inflate.cpp, hd_deflate.cpp) do their
// table work per connection, and connections are independent, so a batch of
// many connections spreads over host threads: one task per connection, or per
// block for the stateless parse.  Threads are started per call (a call is
// a whole batch) and only when there are enough tasks to pay for them.
// NGHTTP2_AMD_HOST_THREADS overrides the count; the default is the hardware
// threads, capped at 16 (the host share of one GPU on the MI355X boxes).
#pragma once

#include <stdlib.h>

#include <algorithm>
#include <atomic>
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

// f(i) for i in [0, n), `grain` consecutive indices per fetch; serial when
// fewer than 2 * grain tasks or one thread.
template <class F>
void parallel_for(size_t n, size_t grain, F &&f) {
  if (grain == 0) grain = 1;
  const size_t chunks = (n + grain - 1) / grain;
  const unsigned t = (unsigned)std::min<size_t>(host_threads(), chunks);
  if (t <= 1) {
    for (size_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (;;) {
      const size_t a = next.fetch_add(grain, std::memory_order_relaxed);
      if (a >= n) return;
      const size_t b = std::min(n, a + grain);
      for (size_t i = a; i < b; ++i) f(i);
    }
  };
  std::vector<std::thread> th;
  th.reserve(t - 1);
  try {
    for (unsigned k = 1; k < t; ++k) th.emplace_back(work);
  } catch (const std::system_error &) {
    // fewer threads than asked: the ones started and this one finish the work
  }
  work();
  for (auto &x : th) x.join();
}

}  // namespace nghttp2_amd_host
