// hd_huff_compat.hip -- link-level drop-in for nghttp2's internal Huffman API
// (lib/nghttp2_hd.h:394-440; reference implementation
// lib/nghttp2_hd_huffman.c:34-147), see include/nghttp2_amd_hd_huffman_compat.h.
//
// Each call is a batch of one string through the batched device API of
// hd_huff.hip (encode_count / encode kernels, and the reference nibble-FSM
// kernel for decode so a chunked string resumes from its carried context).
// One process-wide engine (stream, device buffers, pinned staging) serves
// all callers under a mutex.
#include <hip/hip_runtime.h>
#include <mutex>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/nghttp2_amd_hd.h"
#include "../../include/nghttp2_amd_hd_huffman_compat.h"

extern "C" int nghttp2_bufs_addb(nghttp2_bufs *bufs, uint8_t b) __attribute__((weak));

namespace {

struct Single {
  std::mutex mu;
  bool ready = false, failed = false;
  hipStream_t st = nullptr;
  uint8_t *d_in = nullptr, *d_out = nullptr, *h_pin = nullptr;
  size_t in_cap = 0, out_cap = 0, pin_cap = 0;
  uint32_t *d_meta = nullptr;  // [0..1] in off, [2..3] out off, [4] status, [5] count
  uint16_t *d_fs = nullptr;
  uint8_t *d_fl = nullptr;
  void *d_ws = nullptr;
  size_t ws = 0;
};

Single &eng() {
  static Single s;
  return s;
}

bool hip_ok(hipError_t e) {
  if (e == hipSuccess) return true;
  fprintf(stderr, "nghttp2_amd_hd (compat): HIP error %s\n", hipGetErrorString(e));
  return false;
}

size_t round16(size_t x) { return (x + 15u) & ~size_t(15); }

// grow device / pinned buffers; all sizes include the 16-byte read padding
bool reserve(Single &s, size_t in_bytes, size_t out_bytes) {
  if (!s.ready) {
    if (s.failed) return false;
    s.failed = true;
    if (!hip_ok(hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking))) return false;
    if (!hip_ok(hipMalloc(&s.d_meta, 64))) return false;
    if (!hip_ok(hipMalloc(&s.d_fs, 16)) || !hip_ok(hipMalloc(&s.d_fl, 16))) return false;
    s.ws = nghttp2_amd_hd_huff_workspace_size(1);
    if (!hip_ok(hipMalloc(&s.d_ws, s.ws)) || !hip_ok(hipMemset(s.d_ws, 0, s.ws))) return false;
    s.failed = false;
    s.ready = true;
  }
  in_bytes = round16(in_bytes) + 32;
  out_bytes = round16(out_bytes) + 32;
  if (in_bytes > s.in_cap) {
    if (s.d_in) (void)hipFree(s.d_in);
    s.d_in = nullptr;
    if (!hip_ok(hipMalloc(&s.d_in, in_bytes))) return false;
    s.in_cap = in_bytes;
  }
  if (out_bytes > s.out_cap) {
    if (s.d_out) (void)hipFree(s.d_out);
    s.d_out = nullptr;
    if (!hip_ok(hipMalloc(&s.d_out, out_bytes))) return false;
    s.out_cap = out_bytes;
  }
  const size_t pin = (in_bytes > out_bytes ? in_bytes : out_bytes) + 64;
  if (pin > s.pin_cap) {
    if (s.h_pin) (void)hipHostFree(s.h_pin);
    s.h_pin = nullptr;
    if (!hip_ok(hipHostMalloc((void **)&s.h_pin, pin, hipHostMallocDefault))) return false;
    s.pin_cap = pin;
  }
  return true;
}

// upload one string and its offsets {0, len}
bool upload(Single &s, const uint8_t *src, size_t len) {
  if (len) memcpy(s.h_pin, src, len);
  memset(s.h_pin + len, 0, 16);
  if (!hip_ok(hipMemcpyAsync(s.d_in, s.h_pin, round16(len) + 16, hipMemcpyHostToDevice, s.st)))
    return false;
  const uint32_t off[2] = {0u, (uint32_t)len};
  return hip_ok(hipMemcpyAsync(s.d_meta, off, sizeof(off), hipMemcpyHostToDevice, s.st));
}

}  // namespace

extern "C" {

// The reference's count cannot fail.  When the engine does (no device, out
// of memory, a string past the uint32 range) the count returned is `len`:
// emit_string then takes the raw form (it uses Huffman only when
// enclen < len, lib/nghttp2_hd.c:1011), a valid literal, never a zero
// length prefix followed by Huffman bytes.
size_t nghttp2_hd_huff_encode_count(const uint8_t *src, size_t len) {
  Single &s = eng();
  std::lock_guard<std::mutex> g(s.mu);
  if (len > 0xFFFFFFF0u || !reserve(s, len, 64) || !upload(s, src, len)) return len;
  uint32_t e = 0;
  if (nghttp2_amd_hd_huff_encode_count_batch(s.d_in, s.d_meta, 1, s.d_meta + 4, s.st) != 0 ||
      !hip_ok(hipMemcpyAsync(&e, s.d_meta + 4, 4, hipMemcpyDeviceToHost, s.st)) ||
      !hip_ok(hipStreamSynchronize(s.st)))
    return len;
  return e;
}

int nghttp2_hd_huff_encode(nghttp2_bufs *bufs, const uint8_t *src, size_t srclen) {
  Single &s = eng();
  std::lock_guard<std::mutex> g(s.mu);
  const size_t bound = nghttp2_amd_hd_huff_encode_bound(srclen, 1);
  if (srclen > 0xFFFFFFF0u || !reserve(s, srclen, bound) || !upload(s, src, srclen))
    return NGHTTP2_AMD_ERR_NOMEM;
  uint32_t eoff[2] = {0, 0};
  if (nghttp2_amd_hd_huff_encode_batch(s.d_in, s.d_meta, 1, s.d_out, s.out_cap, s.d_meta + 2,
                                       s.d_ws, s.ws, s.st) != 0 ||
      !hip_ok(hipMemcpyAsync(eoff, s.d_meta + 2, 8, hipMemcpyDeviceToHost, s.st)) ||
      !hip_ok(hipStreamSynchronize(s.st)))
    return NGHTTP2_AMD_ERR_NOMEM;
  const size_t E = eoff[1];
  if (E && (!hip_ok(hipMemcpyAsync(s.h_pin, s.d_out, E, hipMemcpyDeviceToHost, s.st)) ||
            !hip_ok(hipStreamSynchronize(s.st))))
    return NGHTTP2_AMD_ERR_NOMEM;
  // Append in order with the reference's spill behaviour
  // (lib/nghttp2_hd_huffman.c:61-93): fill the current chain buffer, then
  // nghttp2_bufs_addb moves to / allocates the next one or fails with
  // NGHTTP2_ERR_BUFFER_ERROR, leaving the bytes written so far in place.
  const uint8_t *p = s.h_pin;
  size_t left = E;
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
  Single &s = eng();
  std::lock_guard<std::mutex> g(s.mu);
  const size_t cap = srclen * 8 / 5 + 1;
  if (srclen > 0xFFFFFFF0u || !reserve(s, srclen, cap) || !upload(s, src, srclen))
    return NGHTTP2_AMD_ERR_NOMEM;
  // scratch in d_meta: [2..3] dst offsets, [4] status; context in d_fs/d_fl
  const uint32_t doff[2] = {0u, (uint32_t)cap};
  uint16_t fs = ctx->fstate;
  uint8_t fl = ctx->flags;
  int32_t st = 0;
  if (!hip_ok(hipMemcpyAsync(s.d_meta + 2, doff, 8, hipMemcpyHostToDevice, s.st)) ||
      !hip_ok(hipMemcpyAsync(s.d_fs + 4, &fs, 2, hipMemcpyHostToDevice, s.st)) ||
      !hip_ok(hipMemcpyAsync(s.d_fl + 4, &fl, 1, hipMemcpyHostToDevice, s.st)) ||
      nghttp2_amd_hd_huff_decode_fsm_batch(s.d_in, s.d_meta, 1, s.d_out, s.d_meta + 2,
                                           (int32_t *)(s.d_meta + 4), s.d_fs, s.d_fl,
                                           s.d_fs + 4, s.d_fl + 4, 0, s.st) != 0 ||
      !hip_ok(hipMemcpyAsync(&st, s.d_meta + 4, 4, hipMemcpyDeviceToHost, s.st)) ||
      !hip_ok(hipMemcpyAsync(&fs, s.d_fs, 2, hipMemcpyDeviceToHost, s.st)) ||
      !hip_ok(hipMemcpyAsync(&fl, s.d_fl, 1, hipMemcpyDeviceToHost, s.st)) ||
      !hip_ok(hipStreamSynchronize(s.st)))
    return NGHTTP2_AMD_ERR_NOMEM;
  if (st < 0) return st;
  // decoded bytes go to buf->last (the caller guarantees srclen*8/5 bytes)
  if (st && (!hip_ok(hipMemcpyAsync(s.h_pin, s.d_out, (size_t)st, hipMemcpyDeviceToHost, s.st)) ||
             !hip_ok(hipStreamSynchronize(s.st))))
    return NGHTTP2_AMD_ERR_NOMEM;
  memcpy(buf->last, s.h_pin, (size_t)st);
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
