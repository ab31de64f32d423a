/*
 * tests/c/compat_latency.c -- per-call latency of the link-level drop-in
 * (nghttp2_hd_huff_encode_count + nghttp2_hd_huff_encode, and
 * nghttp2_hd_huff_decode with fin=1, as emit_string and hd_inflate_read_huff
 * call them: lib/nghttp2_hd.c:1009/:1037, :1737) against the CPU port of
 * lib/nghttp2_hd_huffman.c (oracle/_build/libhuff_oracle.so, loaded with
 * dlopen: test infrastructure, the checker and the baseline only).
 *
 * Usage: compat_latency <oracle.so> [strings]   -> one JSON line on stdout.
 * Strings are config-2 shaped (8..64 bytes of the pseudo-header alphabet,
 * xorshift64, fixed seed); every engine result is compared with the port's.
 * The count and the encode after it are timed apart (the engine's count runs
 * the whole encode and keeps it, so the encode of the same bytes takes no
 * GPU round trip); then four host threads run the same calls concurrently
 * (one engine per thread), every result compared with the port's.
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "nghttp2_amd_hd_huffman_compat.h"

/* the engine binds nghttp2_bufs_addb weakly; one chain buffer is enough here */
int nghttp2_bufs_addb(nghttp2_bufs *bufs, uint8_t b) {
  (void)bufs;
  (void)b;
  return -502;
}

typedef size_t (*count_fn)(const uint8_t *, size_t);
typedef int (*enc_fn)(uint8_t *, size_t, const uint8_t *, size_t, size_t *);
typedef struct {
  uint16_t fstate;
  uint8_t flags;
} orc_ctx;
typedef void (*init_fn)(orc_ctx *);
typedef long (*dec_fn)(orc_ctx *, uint8_t *, size_t *, const uint8_t *, size_t, int);
typedef int (*oinit_fn)(void);

typedef struct {
  const uint8_t *raw, *enc;
  const size_t *rlen, *eoff;
  int lo, hi, bad;
} job_t;

static void *worker(void *arg);

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(int argc, char **argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s <libhuff_oracle.so> [strings]\n", argv[0]);
    return 2;
  }
  const int n = argc > 2 ? atoi(argv[2]) : 2000;
  void *h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    fprintf(stderr, "dlopen: %s\n", dlerror());
    return 2;
  }
  oinit_fn o_init = (oinit_fn)dlsym(h, "orc_init");
  count_fn o_count = (count_fn)dlsym(h, "orc_encode_count");
  enc_fn o_enc = (enc_fn)dlsym(h, "orc_encode");
  init_fn o_dinit = (init_fn)dlsym(h, "orc_decode_context_init");
  dec_fn o_dec = (dec_fn)dlsym(h, "orc_decode");
  if (!o_init || !o_count || !o_enc || !o_dinit || !o_dec) {
    fprintf(stderr, "oracle symbols missing\n");
    return 2;
  }
  o_init();
  static const char alpha[] = "abcdefghijklmnopqrstuvwxyz0123456789/:._-?=&%ABCDEFGHIJKLMNOPQRSTUVWXYZ";
  uint64_t x = 0x5EED0002ull;
  uint8_t *raw = malloc((size_t)n * 64), *enc = malloc((size_t)n * 256), *dec = malloc(256);
  size_t *rlen = malloc(sizeof(size_t) * n), *eoff = malloc(sizeof(size_t) * (n + 1));
  for (int i = 0; i < n; ++i) {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    rlen[i] = 8 + x % 57;
    for (size_t k = 0; k < rlen[i]; ++k) {
      x ^= x << 13, x ^= x >> 7, x ^= x << 17;
      raw[(size_t)i * 64 + k] = (uint8_t)alpha[x % (sizeof(alpha) - 1)];
    }
  }
  size_t raw_total = 0;
  for (int i = 0; i < n; ++i) raw_total += rlen[i];
  /* port: count + encode, decode */
  size_t total = 0;
  eoff[0] = 0;
  double t0 = now();
  for (int i = 0; i < n; ++i) {
    size_t w = 0;
    const size_t c = o_count(raw + (size_t)i * 64, rlen[i]);
    o_enc(enc + eoff[i], 256, raw + (size_t)i * 64, rlen[i], &w);
    eoff[i + 1] = eoff[i] + w;
    total += c;
  }
  const double port_enc = (now() - t0) / n;
  t0 = now();
  for (int i = 0; i < n; ++i) {
    orc_ctx c;
    size_t w = 0;
    o_dinit(&c);
    o_dec(&c, dec, &w, enc + eoff[i], eoff[i + 1] - eoff[i], 1);
  }
  const double port_dec = (now() - t0) / n;
  /* engine: warm up (stream, buffers), then time */
  int bad = 0;
  uint8_t *ebuf = malloc(512);
  for (int pass = 0; pass < 2; ++pass) {
    double te = 0, td = 0, tc = 0;
    for (int i = 0; i < n; ++i) {
      nghttp2_buf_chain ch;
      memset(&ch, 0, sizeof(ch));
      ch.buf.begin = ch.buf.pos = ch.buf.last = ch.buf.mark = ebuf;
      ch.buf.end = ebuf + 512;
      nghttp2_bufs b;
      memset(&b, 0, sizeof(b));
      b.head = b.cur = &ch;
      b.chunk_length = 512;
      b.max_chunk = 1;
      b.chunk_used = 1;
      double a = now();
      const size_t c = nghttp2_hd_huff_encode_count(raw + (size_t)i * 64, rlen[i]);
      const double a2 = now();
      const int rv = nghttp2_hd_huff_encode(&b, raw + (size_t)i * 64, rlen[i]);
      te += now() - a;
      tc += a2 - a;
      const size_t E = (size_t)(ch.buf.last - ebuf);
      if (rv != 0 || c != E || E != eoff[i + 1] - eoff[i] || memcmp(ebuf, enc + eoff[i], E) != 0) ++bad;
      nghttp2_hd_huff_decode_context ctx;
      nghttp2_buf ob;
      ob.begin = ob.pos = ob.last = ob.mark = dec;
      ob.end = dec + 256;
      a = now();
      nghttp2_hd_huff_decode_context_init(&ctx);
      const nghttp2_ssize d = nghttp2_hd_huff_decode(&ctx, &ob, ebuf, E, 1);
      td += now() - a;
      if (d != (nghttp2_ssize)E || (size_t)(ob.last - dec) != rlen[i] ||
          memcmp(dec, raw + (size_t)i * 64, rlen[i]) != 0)
        ++bad;
    }
    if (pass == 1) {
      /* four host threads, one engine each, a quarter of the strings each */
      pthread_t th[4];
      job_t jobs[4];
      const double w0 = now();
      for (int k = 0; k < 4; ++k) {
        jobs[k].raw = raw, jobs[k].enc = enc, jobs[k].rlen = rlen, jobs[k].eoff = eoff;
        jobs[k].lo = n * k / 4, jobs[k].hi = n * (k + 1) / 4, jobs[k].bad = 0;
        pthread_create(&th[k], NULL, worker, &jobs[k]);
      }
      int tbad = 0;
      for (int k = 0; k < 4; ++k) {
        pthread_join(th[k], NULL);
        tbad += jobs[k].bad;
      }
      const double wall4 = now() - w0;
      bad += tbad;
      printf("{\"strings\": %d, \"raw_bytes\": %zu, \"enc_bytes\": %zu, "
             "\"engine_encode_us_per_call\": %.2f, \"engine_count_us_per_call\": %.2f, "
             "\"engine_encode_after_count_us_per_call\": %.2f, \"engine_decode_us_per_call\": %.2f, "
             "\"port_encode_us_per_call\": %.4f, \"port_decode_us_per_call\": %.4f, "
             "\"threads4_us_per_string\": %.2f, \"threads4_mismatches\": %d, "
             "\"mismatches\": %d}\n",
             n, raw_total, total, 1e6 * te / n, 1e6 * tc / n, 1e6 * (te - tc) / n, 1e6 * td / n,
             1e6 * port_enc, 1e6 * port_dec, 1e6 * wall4 / n, tbad, bad);
    }
  }
  return bad ? 1 : 0;
}

/* one host thread: count + encode + decode of its strings through its own
 * engine, each result against the port's */
static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  uint8_t ebuf[512], dec[256];
  for (int i = j->lo; i < j->hi; ++i) {
    const uint8_t *r = j->raw + (size_t)i * 64;
    nghttp2_buf_chain ch;
    memset(&ch, 0, sizeof(ch));
    ch.buf.begin = ch.buf.pos = ch.buf.last = ch.buf.mark = ebuf;
    ch.buf.end = ebuf + sizeof ebuf;
    nghttp2_bufs b;
    memset(&b, 0, sizeof(b));
    b.head = b.cur = &ch;
    b.chunk_length = sizeof ebuf;
    b.max_chunk = 1;
    b.chunk_used = 1;
    const size_t c = nghttp2_hd_huff_encode_count(r, j->rlen[i]);
    const int rv = nghttp2_hd_huff_encode(&b, r, j->rlen[i]);
    const size_t E = (size_t)(ch.buf.last - ebuf);
    if (rv != 0 || c != E || E != j->eoff[i + 1] - j->eoff[i] || memcmp(ebuf, j->enc + j->eoff[i], E) != 0)
      ++j->bad;
    nghttp2_hd_huff_decode_context ctx;
    nghttp2_buf ob;
    ob.begin = ob.pos = ob.last = ob.mark = dec;
    ob.end = dec + sizeof dec;
    nghttp2_hd_huff_decode_context_init(&ctx);
    const nghttp2_ssize d = nghttp2_hd_huff_decode(&ctx, &ob, ebuf, E, 1);
    if (d != (nghttp2_ssize)E || (size_t)(ob.last - dec) != j->rlen[i] || memcmp(dec, r, j->rlen[i]) != 0)
      ++j->bad;
  }
  return NULL;
}
