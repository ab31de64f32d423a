// hd_sharded.cpp -- one batch over several GPUs, behind
// include/nghttp2_amd_hd.h "nghttp2_amd_hd_sharded_*".
//
// Header strings are independent (lib/nghttp2_hd_huffman.c encodes and
// decodes each string on its own), so a batch cuts into contiguous string
// ranges balanced by bytes, one per device, and nothing is exchanged between
// devices: no RCCL collective, xGMI unused.  Each shard has a worker thread
// that owns its device context (stream, buffers, workspace) for the engine's
// lifetime -- the reference's one-session-per-thread model
// (doc/programmers-guide.rst:35-40) with a GPU behind each thread.
//
// A host-resident call runs in two phases per shard: (1) H2D of the shard's
// bytes and offsets, the engine kernels, D2H of its output total; (2) after
// the caller has summed the totals into the shards' merged bases, D2H of
// the shard's output straight to its merged position, offsets rebased on
// the host.  The shard's offsets go to the device as they are (absolute in
// the caller's pool): the kernels get a source pointer moved back by the
// shard's first 16-byte chunk, so src + off[i] lands in the shard's copy.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/nghttp2_amd_hd.h"

namespace {

bool hip_ok(hipError_t e) {
  if (e == hipSuccess) return true;
  fprintf(stderr, "nghttp2_amd_hd (sharded): HIP error %s\n", hipGetErrorString(e));
  return false;
}

size_t round16(size_t x) { return (x + 15u) & ~size_t(15); }

// A device buffer that grows (never shrinks) on its context's device.
struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  bool reserve(size_t need) {
    if (need <= cap) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    need = round16(need) + 256;
    if (!hip_ok(hipMalloc(&p, need))) return false;
    cap = need;
    return true;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T *as() const { return static_cast<T *>(p); }
};

// One shard's device context and worker thread.  The worker runs one job at
// a time; run() hands it a job, wait() joins it.
struct Shard {
  int device = 0;
  hipStream_t st = nullptr;
  DevBuf src, src_off, dst, dst_off, status, fstate, flags, ws;
  std::thread th;
  std::mutex mu;
  std::condition_variable cv, done_cv;
  std::function<void()> job;
  bool has_job = false, busy = false, quit = false;
  int init_rv = 0;

  void loop() {
    init_rv = hip_ok(hipSetDevice(device)) && hip_ok(hipStreamCreateWithFlags(&st, hipStreamNonBlocking))
                  ? 0
                  : NGHTTP2_AMD_ERR_FATAL;
    {
      std::lock_guard<std::mutex> l(mu);
      busy = false;
    }
    done_cv.notify_all();
    for (;;) {
      std::function<void()> j;
      {
        std::unique_lock<std::mutex> l(mu);
        cv.wait(l, [&] { return has_job || quit; });
        if (quit) break;
        j = std::move(job);
        has_job = false;
      }
      j();
      {
        std::lock_guard<std::mutex> l(mu);
        busy = false;
      }
      done_cv.notify_all();
    }
    for (DevBuf *b : {&src, &src_off, &dst, &dst_off, &status, &fstate, &flags, &ws}) b->release();
    if (st) (void)hipStreamDestroy(st);
  }
  void run(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> l(mu);
      job = std::move(f);
      has_job = true;
      busy = true;
    }
    cv.notify_one();
  }
  void wait() {
    std::unique_lock<std::mutex> l(mu);
    done_cv.wait(l, [&] { return !busy; });
  }
};

}  // namespace

struct nghttp2_amd_hd_sharded {
  std::vector<Shard *> shards;
};

namespace {

// every shard runs f(k); returns when all have finished
void run_all(nghttp2_amd_hd_sharded *s, const std::function<void(uint32_t)> &f) {
  const uint32_t m = (uint32_t)s->shards.size();
  for (uint32_t k = 0; k < m; ++k) s->shards[k]->run([&f, k] { f(k); });
  for (uint32_t k = 0; k < m; ++k) s->shards[k]->wait();
}

int first_error(const std::vector<int> &rv) {
  for (int r : rv)
    if (r != 0) return r;
  return 0;
}

// byte-balanced cuts (the first string starting at or after each share)
void cut(const uint32_t *off, uint32_t n, uint32_t m, uint32_t *cuts) {
  const uint64_t base = off[0], total = (uint64_t)off[n] - off[0];
  cuts[0] = 0;
  for (uint32_t r = 1; r < m; ++r) {
    const uint64_t target = base + total * r / m;
    const uint32_t *p = std::lower_bound(off, off + n, (uint32_t)target);
    cuts[r] = std::max(cuts[r - 1], (uint32_t)(p - off));
  }
  cuts[m] = n;
}

// Host-resident shard, phase 1: upload and run; returns the output total.
// DEC: decode (decode_batch_auto) else encode (encode_batch).
template <bool DEC>
int shard_phase1(Shard &sh, const uint8_t *src, const uint32_t *off, uint32_t s0, uint32_t s1,
                 bool want_ctx, uint64_t *total) {
  if (!hip_ok(hipSetDevice(sh.device))) return NGHTTP2_AMD_ERR_FATAL;
  const uint32_t n = s1 - s0;
  const uint64_t a = off[s0], b = off[s1];
  const uint64_t a16 = a & ~(uint64_t)15;
  const uint64_t bytes = round16(b) + 16 - a16;  // the padding every pool read may touch
  const uint64_t in_bytes = b - a;
  const size_t out_cap = DEC ? nghttp2_amd_hd_huff_decode_bound(in_bytes, n)
                             : nghttp2_amd_hd_huff_encode_bound(in_bytes, n);
  const size_t wsz = nghttp2_amd_hd_huff_workspace_size(n);
  if (!sh.src.reserve(bytes) || !sh.src_off.reserve(4ull * (n + 1)) || !sh.dst.reserve(out_cap) ||
      !sh.dst_off.reserve(4ull * (n + 1)) || !sh.ws.reserve(wsz) ||
      (DEC && !sh.status.reserve(4ull * std::max(1u, n))) ||
      (DEC && want_ctx && (!sh.fstate.reserve(2ull * std::max(1u, n)) || !sh.flags.reserve(std::max(1u, n)))))
    return NGHTTP2_AMD_ERR_NOMEM;
  if (!hip_ok(hipMemcpyAsync(sh.src.p, src + a16, bytes, hipMemcpyHostToDevice, sh.st)) ||
      !hip_ok(hipMemcpyAsync(sh.src_off.p, off + s0, 4ull * (n + 1), hipMemcpyHostToDevice, sh.st)))
    return NGHTTP2_AMD_ERR_FATAL;
  // the kernels address src + off[i]: a base moved back by the shard's first chunk
  const uint8_t *ksrc = sh.src.as<uint8_t>() - a16;
  int rv;
  if (DEC)
    rv = nghttp2_amd_hd_huff_decode_batch_auto(ksrc, sh.src_off.as<uint32_t>(), n, in_bytes,
                                               sh.dst.as<uint8_t>(), out_cap, sh.dst_off.as<uint32_t>(),
                                               sh.status.as<int32_t>(),
                                               want_ctx ? sh.fstate.as<uint16_t>() : nullptr,
                                               want_ctx ? sh.flags.as<uint8_t>() : nullptr, sh.st);
  else
    rv = nghttp2_amd_hd_huff_encode_batch(ksrc, sh.src_off.as<uint32_t>(), n, sh.dst.as<uint8_t>(),
                                          out_cap, sh.dst_off.as<uint32_t>(), sh.ws.p, sh.ws.cap, sh.st);
  if (rv != 0) return rv;
  uint32_t t = 0;
  if (!hip_ok(hipMemcpyAsync(&t, sh.dst_off.as<uint32_t>() + n, 4, hipMemcpyDeviceToHost, sh.st)) ||
      !hip_ok(hipStreamSynchronize(sh.st)))
    return NGHTTP2_AMD_ERR_FATAL;
  *total = t;  // (encode: NGHTTP2_AMD_OFF_OVERFLOW when the shard overflowed)
  return 0;
}

// phase 2: the shard's output to dst + base, its offsets (and per-string
// results) to their merged places, rebased on the host
template <bool DEC>
int shard_phase2(Shard &sh, uint32_t s0, uint32_t s1, bool last, uint64_t base, uint64_t total,
                 uint8_t *dst, uint32_t *dst_off, int32_t *status, uint16_t *fstate, uint8_t *flags) {
  if (!hip_ok(hipSetDevice(sh.device))) return NGHTTP2_AMD_ERR_FATAL;
  const uint32_t n = s1 - s0;
  const uint32_t noff = last ? n + 1 : n;  // (shard k's dst_off[n] is shard k+1's dst_off[0])
  if ((total && !hip_ok(hipMemcpyAsync(dst + base, sh.dst.p, total, hipMemcpyDeviceToHost, sh.st))) ||
      (noff && !hip_ok(hipMemcpyAsync(dst_off + s0, sh.dst_off.p, 4ull * noff, hipMemcpyDeviceToHost, sh.st))))
    return NGHTTP2_AMD_ERR_FATAL;
  if (DEC && n) {
    if (!hip_ok(hipMemcpyAsync(status + s0, sh.status.p, 4ull * n, hipMemcpyDeviceToHost, sh.st)) ||
        (fstate && !hip_ok(hipMemcpyAsync(fstate + s0, sh.fstate.p, 2ull * n, hipMemcpyDeviceToHost, sh.st))) ||
        (flags && !hip_ok(hipMemcpyAsync(flags + s0, sh.flags.p, n, hipMemcpyDeviceToHost, sh.st))))
      return NGHTTP2_AMD_ERR_FATAL;
  }
  if (!hip_ok(hipStreamSynchronize(sh.st))) return NGHTTP2_AMD_ERR_FATAL;
  const uint32_t b32 = (uint32_t)base;
  for (uint32_t i = 0; i < noff; ++i) dst_off[s0 + i] += b32;
  return 0;
}

template <bool DEC>
int sharded_host(nghttp2_amd_hd_sharded *s, const uint8_t *src, const uint32_t *src_off, uint32_t n,
                 uint8_t *dst, size_t dst_cap, uint32_t *dst_off, int32_t *status, uint16_t *fstate,
                 uint8_t *flags) {
  if (!s || !dst_off) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (n && (!src || !src_off || !dst || (DEC && !status))) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (DEC && (fstate == nullptr) != (flags == nullptr)) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (n == 0) {
    dst_off[0] = 0;
    return 0;
  }
  for (uint32_t i = 0; i < n; ++i)  // a descending pair would cut shards wrongly
    if (src_off[i + 1] < src_off[i]) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  const uint32_t m = (uint32_t)s->shards.size();
  std::vector<uint32_t> cuts(m + 1);
  cut(src_off, n, m, cuts.data());
  std::vector<int> rv(m, 0);
  std::vector<uint64_t> tot(m, 0);
  run_all(s, [&](uint32_t k) {
    if (cuts[k + 1] > cuts[k] || k + 1 == m)
      rv[k] = shard_phase1<DEC>(*s->shards[k], src, src_off, cuts[k], cuts[k + 1], fstate != nullptr, &tot[k]);
  });
  if (const int e = first_error(rv)) return e;
  std::vector<uint64_t> base(m, 0);
  uint64_t sum = 0;
  bool over = false;
  for (uint32_t k = 0; k < m; ++k) {
    if (!DEC && tot[k] == NGHTTP2_AMD_OFF_OVERFLOW) over = true;
    base[k] = sum;
    sum += tot[k];
  }
  if (over || sum > dst_cap || sum > 0xFFFFFFFEull) {
    if (!DEC) dst_off[n] = NGHTTP2_AMD_OFF_OVERFLOW;
    return NGHTTP2_AMD_ERR_BUFFER_ERROR;
  }
  run_all(s, [&](uint32_t k) {
    if (cuts[k + 1] > cuts[k] || k + 1 == m)
      rv[k] = shard_phase2<DEC>(*s->shards[k], cuts[k], cuts[k + 1], k + 1 == m, base[k], tot[k], dst,
                                dst_off, status, fstate, flags);
  });
  return first_error(rv);
}

template <bool DEC>
int sharded_dev(nghttp2_amd_hd_sharded *s, nghttp2_amd_hd_shard *sh) {
  if (!s || !sh) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  const uint32_t m = (uint32_t)s->shards.size();
  run_all(s, [&](uint32_t k) {
    nghttp2_amd_hd_shard &x = sh[k];
    Shard &c = *s->shards[k];
    x.out_bytes = 0;
    if (!hip_ok(hipSetDevice(c.device))) {
      x.rv = NGHTTP2_AMD_ERR_FATAL;
      return;
    }
    if (DEC) {
      x.rv = nghttp2_amd_hd_huff_decode_batch_auto(x.src, x.src_off, x.n, x.in_bytes, x.dst, x.dst_cap,
                                                   x.dst_off, x.status, x.fstate, x.flags, c.st);
    } else {
      const size_t wsz = nghttp2_amd_hd_huff_workspace_size(x.n);
      x.rv = c.ws.reserve(wsz) ? nghttp2_amd_hd_huff_encode_batch(x.src, x.src_off, x.n, x.dst, x.dst_cap,
                                                                  x.dst_off, c.ws.p, c.ws.cap, c.st)
                               : NGHTTP2_AMD_ERR_NOMEM;
    }
    uint32_t t = 0;
    if (x.rv == 0 && (!hip_ok(hipMemcpyAsync(&t, x.dst_off + x.n, 4, hipMemcpyDeviceToHost, c.st)) ||
                      !hip_ok(hipStreamSynchronize(c.st))))
      x.rv = NGHTTP2_AMD_ERR_FATAL;
    x.out_bytes = t;
  });
  uint64_t sum = 0;
  int e = 0;
  for (uint32_t k = 0; k < m; ++k) {
    sh[k].out_base = sum;
    sum += sh[k].out_bytes;
    if (!e && sh[k].rv) e = sh[k].rv;
  }
  return e;
}

}  // namespace

extern "C" {

int nghttp2_amd_hd_shard_bounds(const uint32_t *off, uint32_t n, uint32_t nshards, uint32_t *cuts) {
  if (!off || !cuts || nshards == 0) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  for (uint32_t i = 0; i < n; ++i)
    if (off[i + 1] < off[i]) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  cut(off, n, nshards, cuts);
  return 0;
}

int nghttp2_amd_hd_sharded_new(nghttp2_amd_hd_sharded **out, const int *devices, uint32_t ndevices) {
  if (!out || !devices || ndevices == 0) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  int count = 0;
  if (!hip_ok(hipGetDeviceCount(&count))) return NGHTTP2_AMD_ERR_FATAL;
  for (uint32_t k = 0; k < ndevices; ++k)
    if (devices[k] < 0 || devices[k] >= count) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  nghttp2_amd_hd_sharded *s = new (std::nothrow) nghttp2_amd_hd_sharded;
  if (!s) return NGHTTP2_AMD_ERR_NOMEM;
  int rv = 0;
  for (uint32_t k = 0; k < ndevices && rv == 0; ++k) {
    Shard *sh = new (std::nothrow) Shard;
    if (!sh) {
      rv = NGHTTP2_AMD_ERR_NOMEM;
      break;
    }
    sh->device = devices[k];
    sh->busy = true;
    try {
      sh->th = std::thread([sh] { sh->loop(); });
    } catch (...) {
      delete sh;
      rv = NGHTTP2_AMD_ERR_NOMEM;
      break;
    }
    s->shards.push_back(sh);
    sh->wait();  // the worker made its stream
    rv = sh->init_rv;
  }
  if (rv != 0) {
    nghttp2_amd_hd_sharded_del(s);
    return rv;
  }
  *out = s;
  return 0;
}

void nghttp2_amd_hd_sharded_del(nghttp2_amd_hd_sharded *s) {
  if (!s) return;
  for (Shard *sh : s->shards) {
    {
      std::lock_guard<std::mutex> l(sh->mu);
      sh->quit = true;
    }
    sh->cv.notify_one();
    if (sh->th.joinable()) sh->th.join();
    delete sh;
  }
  delete s;
}

uint32_t nghttp2_amd_hd_sharded_count(const nghttp2_amd_hd_sharded *s) {
  return s ? (uint32_t)s->shards.size() : 0u;
}

int nghttp2_amd_hd_sharded_encode(nghttp2_amd_hd_sharded *s, const uint8_t *src, const uint32_t *src_off,
                                  uint32_t n, uint8_t *dst, size_t dst_cap, uint32_t *dst_off) {
  return sharded_host<false>(s, src, src_off, n, dst, dst_cap, dst_off, nullptr, nullptr, nullptr);
}

int nghttp2_amd_hd_sharded_decode(nghttp2_amd_hd_sharded *s, const uint8_t *src, const uint32_t *src_off,
                                  uint32_t n, uint8_t *dst, size_t dst_cap, uint32_t *dst_off,
                                  int32_t *status, uint16_t *fstate, uint8_t *flags) {
  return sharded_host<true>(s, src, src_off, n, dst, dst_cap, dst_off, status, fstate, flags);
}

int nghttp2_amd_hd_sharded_encode_dev(nghttp2_amd_hd_sharded *s, nghttp2_amd_hd_shard *shards) {
  return sharded_dev<false>(s, shards);
}

int nghttp2_amd_hd_sharded_decode_dev(nghttp2_amd_hd_sharded *s, nghttp2_amd_hd_shard *shards) {
  return sharded_dev<true>(s, shards);
}

}  // extern "C"
