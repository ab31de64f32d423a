// hd_huff_compat.hip -- link-level drop-in for nghttp2's internal Huffman API
// (lib/nghttp2_hd.h:394-440; reference implementation
// lib/nghttp2_hd_huffman.c:34-147), see include/nghttp2_amd_hd_huffman_compat.h.
//
// Each call is a batch of one string through the batched device API of
// hd_huff.hip (encode_count / encode kernels, and the reference nibble-FSM
// kernel for decode so a chunked string resumes from its carried context).
//
// Threading follows nghttp2's model (doc/programmers-guide.rst:35-40: one
// session per thread, nothing shared): every calling host thread gets its
// own engine -- HIP stream, a mapped pinned block, device workspace -- on the
// device current in that thread at its first call, so concurrent callers
// never serialise on a lock or a stream.  A call is one round trip without
// copies: the kernels read the string and its metadata from the mapped
// block and write the results and output bytes into it (round 5: an H2D and
// a D2H copy around the kernels took 21.0 / 26.7 us per encode pair /
// decode), then one synchronisation.
//
// Strings of kCopyMin bytes or more go the other way: the block is copied to
// a device buffer, the kernels run there and the results are copied back --
// for long strings one DMA copy each way beats many waves reading and writing
// uncached host memory across PCIe (round 6, advisor).
//
// emit_string (lib/nghttp2_hd.c:1009, :1037) asks for the count and then,
// when Huffman wins, for the encoding of the same bytes.  The count runs the
// whole encode and keeps its output (and a copy of the input) in the
// thread's engine; an encode of the same bytes right after it takes the kept
// output without a second round trip (its input is compared byte for byte,
// so a caller that changed the bytes in between gets a fresh encode).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <new>
#include <vector>

#include "../../include/nghttp2_amd_hd.h"
#include "../../include/nghttp2_amd_hd_huffman_compat.h"

extern "C" int nghttp2_bufs_addb(nghttp2_bufs *bufs, uint8_t b) __attribute__((weak));

namespace {

bool hip_ok(hipError_t e) {
  if (e == hipSuccess) return true;
  fprintf(stderr, "nghttp2_amd_hd (compat): HIP error %s\n", hipGetErrorString(e));
  return false;
}

size_t round16(size_t x) { return (x + 15u) & ~size_t(15); }

constexpr size_t kCopyMin = 64u << 10;  // string bytes from which a call copies instead of mapping

// Layout of one call (device buffer and pinned block alike):
//   [in: string bytes, round16(len) + 16][meta: 64 B][res: 16 B][out bytes]
// meta: u32 src_off[2] | u32 dst_off[2] | u16 init fstate | u8 init flags
// res:  encode: u32 enc_off[2];  decode: i32 status | u16 fstate | u8 flags
struct Layout {
  size_t meta, res, out, total;
  Layout(size_t len, size_t out_cap) {
    meta = round16(len) + 16;
    res = meta + 64;
    out = res + 16;
    total = out + round16(out_cap) + 16;
  }
};

struct Engine {
  bool ready = false;
  int device = -1;
  hipStream_t st = nullptr;
  uint8_t *d_buf = nullptr, *h_pin = nullptr;  // d_buf: h_pin's device address
  size_t cap = 0;
  uint8_t *d_dev = nullptr;  // long strings: a device copy of the block
  size_t dev_cap = 0;
  void *d_ws = nullptr;
  size_t ws = 0;
  // the last count's full encode (emit_string's count -> encode pair)
  bool kept = false;
  std::vector<uint8_t> kept_src, kept_out;

  ~Engine() { release(); }
  void release() {
    if (h_pin) (void)hipHostFree(h_pin);
    if (d_dev) (void)hipFree(d_dev);
    if (d_ws) (void)hipFree(d_ws);
    if (st) (void)hipStreamDestroy(st);
    d_buf = h_pin = d_dev = nullptr;
    d_ws = nullptr;
    st = nullptr;
    cap = ws = dev_cap = 0;
    ready = false;
  }
  // the thread's stream and buffers on its current device; grows to `need`
  bool reserve(size_t need) {
    int dev = 0;
    if (!hip_ok(hipGetDevice(&dev))) return false;
    if (ready && dev != device) {  // the thread moved to another device
      this->~Engine();
      new (this) Engine();
    }
    if (!ready) {
      // (a failed init releases what it made: a thread whose allocations
      // keep failing does not leak a stream per call)
      device = dev;
      if (!hip_ok(hipStreamCreateWithFlags(&st, hipStreamNonBlocking))) {
        st = nullptr;
        return false;
      }
      ws = nghttp2_amd_hd_huff_workspace_size(1);
      if (!hip_ok(hipMalloc(&d_ws, ws))) {
        d_ws = nullptr;
        release();
        return false;
      }
      ready = true;
    }
    if (need > cap) {
      need = round16(need) + 4096;
      if (h_pin) (void)hipHostFree(h_pin);
      d_buf = nullptr;
      h_pin = nullptr;
      cap = 0;
      if (!hip_ok(hipHostMalloc((void **)&h_pin, need, hipHostMallocMapped | hipHostMallocCoherent)))
        return false;
      if (!hip_ok(hipHostGetDevicePointer((void **)&d_buf, h_pin, 0))) {
        (void)hipHostFree(h_pin);
        h_pin = nullptr;
        return false;
      }
      cap = need;
    }
    return true;
  }
  // The block the kernels of a call use: the mapped pinned block, or (a
  // string of kCopyMin bytes or more) a device buffer that receives the
  // block's input and metadata [0, res) by one copy.
  uint8_t *stage(const Layout &l, size_t len) {
    if (len < kCopyMin) return d_buf;
    if (l.total > dev_cap) {
      if (d_dev) (void)hipFree(d_dev);
      d_dev = nullptr;
      dev_cap = 0;
      if (!hip_ok(hipMalloc((void **)&d_dev, l.total))) return nullptr;
      dev_cap = l.total;
    }
    if (!hip_ok(hipMemcpyAsync(d_dev, h_pin, l.res, hipMemcpyHostToDevice, st))) return nullptr;
    return d_dev;
  }
  // after the kernels: the results and output back into the pinned block
  // (copied calls), then the one synchronisation
  bool finish(const Layout &l, const uint8_t *d) {
    if (d != d_buf &&
        !hip_ok(hipMemcpyAsync(h_pin + l.res, d + l.res, l.total - l.res, hipMemcpyDeviceToHost, st)))
      return false;
    return hip_ok(hipStreamSynchronize(st));
  }
};

Engine &eng() {
  static thread_local Engine e;
  return e;
}

// the string (zero padded) into the mapped block, ahead of its metadata
void upload(Engine &e, const Layout &l, const uint8_t *src, size_t len) {
  if (len) memcpy(e.h_pin, src, len);
  memset(e.h_pin + len, 0, l.meta - len);
}

// the whole encode of one string: the kept output on success
bool encode_one(Engine &e, const uint8_t *src, size_t len) {
  e.kept = false;
  const size_t bound = nghttp2_amd_hd_huff_encode_bound(len, 1);
  const Layout l(len, bound);
  if (len > 0xFFFFFFF0u || !e.reserve(l.total)) return false;
  uint32_t *m = reinterpret_cast<uint32_t *>(e.h_pin + l.meta);
  m[0] = 0;
  m[1] = (uint32_t)len;
  upload(e, l, src, len);
  uint8_t *d = e.stage(l, len);
  if (!d) return false;
  if (nghttp2_amd_hd_huff_encode_batch(d, reinterpret_cast<const uint32_t *>(d + l.meta), 1, d + l.out,
                                       l.total - l.out, reinterpret_cast<uint32_t *>(d + l.res), e.d_ws,
                                       e.ws, e.st) != 0 ||
      !e.finish(l, d))
    return false;
  const uint32_t *r = reinterpret_cast<const uint32_t *>(e.h_pin + l.res);
  if (r[1] > bound) return false;
  e.kept_src.assign(src, src + len);
  e.kept_out.assign(e.h_pin + l.out, e.h_pin + l.out + r[1]);
  e.kept = true;
  return true;
}

}  // namespace

extern "C" {

// The reference's count cannot fail.  When the engine does (no device, out
// of memory, a string past the uint32 range) the count returned is `len`:
// emit_string then takes the raw form (it uses Huffman only when
// enclen < len, lib/nghttp2_hd.c:1011), a valid literal, never a zero
// length prefix followed by Huffman bytes.
size_t nghttp2_hd_huff_encode_count(const uint8_t *src, size_t len) {
  Engine &e = eng();
  if (!encode_one(e, src, len)) return len;
  return e.kept_out.size();
}

int nghttp2_hd_huff_encode(nghttp2_bufs *bufs, const uint8_t *src, size_t srclen) {
  Engine &e = eng();
  const bool hit = e.kept && e.kept_src.size() == srclen &&
                   (srclen == 0 || memcmp(e.kept_src.data(), src, srclen) == 0);
  if (!hit && !encode_one(e, src, srclen)) return NGHTTP2_AMD_ERR_NOMEM;
  e.kept = false;  // one encode per count
  // Append in order with the reference's spill behaviour
  // (lib/nghttp2_hd_huffman.c:61-93): fill the current chain buffer, then
  // nghttp2_bufs_addb moves to / allocates the next one or fails with
  // NGHTTP2_ERR_BUFFER_ERROR, leaving the bytes written so far in place.
  const uint8_t *p = e.kept_out.data();
  size_t left = e.kept_out.size();
  while (left) {
    nghttp2_buf *cur = &bufs->cur->buf;
    size_t avail = (size_t)(cur->end - cur->last);
    if (avail) {
      const size_t k = avail < left ? avail : left;
      memcpy(cur->last, p, k);
      cur->last += k;
      p += k;
      left -= k;
      continue;
    }
    if (!nghttp2_bufs_addb) return NGHTTP2_AMD_ERR_BUFFER_ERROR;
    const int rv = nghttp2_bufs_addb(bufs, *p);
    if (rv != 0) return rv;
    ++p;
    --left;
  }
  return 0;
}

void nghttp2_hd_huff_decode_context_init(nghttp2_hd_huff_decode_context *ctx) {
  // lib/nghttp2_hd_huffman.c:106-109
  ctx->fstate = 0;
  ctx->flags = NGHTTP2_AMD_HUFF_ACCEPTED;
}

nghttp2_ssize nghttp2_hd_huff_decode(nghttp2_hd_huff_decode_context *ctx, nghttp2_buf *buf,
                                     const uint8_t *src, size_t srclen, int fin) {
  Engine &e = eng();
  const size_t cap = srclen * 8 / 5 + 1;
  const Layout l(srclen, cap);
  if (srclen > 0xFFFFFFF0u || !e.reserve(l.total)) return NGHTTP2_AMD_ERR_NOMEM;
  uint8_t *m = e.h_pin + l.meta;
  const uint32_t offs[4] = {0u, (uint32_t)srclen, 0u, (uint32_t)cap};
  memcpy(m, offs, sizeof offs);
  memcpy(m + 16, &ctx->fstate, 2);
  m[18] = ctx->flags;
  upload(e, l, src, srclen);
  uint8_t *d = e.stage(l, srclen);
  if (!d) return NGHTTP2_AMD_ERR_NOMEM;
  const uint32_t *dm = reinterpret_cast<const uint32_t *>(d + l.meta);
  if (nghttp2_amd_hd_huff_decode_fsm_batch(d, dm, 1, d + l.out, dm + 2, reinterpret_cast<int32_t *>(d + l.res),
                                           reinterpret_cast<uint16_t *>(d + l.res + 4), d + l.res + 6,
                                           reinterpret_cast<const uint16_t *>(d + l.meta + 16),
                                           d + l.meta + 18, 0, e.st) != 0 ||
      !e.finish(l, d))
    return NGHTTP2_AMD_ERR_NOMEM;
  int32_t st;
  uint16_t fs;
  memcpy(&st, e.h_pin + l.res, 4);
  memcpy(&fs, e.h_pin + l.res + 4, 2);
  const uint8_t fl = e.h_pin[l.res + 6];
  if (st < 0) return st;
  // decoded bytes go to buf->last (the caller guarantees srclen*8/5 bytes)
  memcpy(buf->last, e.h_pin + l.out, (size_t)st);
  buf->last += st;
  // lib/nghttp2_hd_huffman.c:135-142
  ctx->fstate = fs;
  ctx->flags = fl;
  if (fin && !(ctx->flags & NGHTTP2_AMD_HUFF_ACCEPTED)) return NGHTTP2_AMD_ERR_HEADER_COMP;
  return (nghttp2_ssize)srclen;
}

int nghttp2_hd_huff_decode_failure_state(nghttp2_hd_huff_decode_context *ctx) {
  // lib/nghttp2_hd_huffman.c:145-147
  return ctx->fstate == NGHTTP2_AMD_HUFF_FAIL_STATE;
}

}  // extern "C"
