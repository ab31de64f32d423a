/*
 * tests/c/test_compat.c -- the reference's Huffman unit tests, replayed in C
 * through the engine's link-level drop-in (libnghttp2_amd_hd.so exports
 * nghttp2_hd_huff_* with the reference's signatures).
 *
 *   test_nghttp2_hd_huff_encode  tests/nghttp2_hd_test.c:1605-1633
 *   test_nghttp2_hd_huff_decode  tests/nghttp2_hd_test.c:1635-1670
 *   plus chain spill (tests/nghttp2_hd_test.c:1367+ deflate_hd_vec relies on
 *   it), wrap-mode overflow (:1322-1365), chunked streaming decode
 *   (tests/nghttp2_test_helper.c:165-205) and RFC 7541 C.4.1.
 *
 * nghttp2_bufs_addb below is a test double with the semantics of
 * lib/nghttp2_buf.c:294-383 (advance to / allocate the next chain buffer,
 * NGHTTP2_ERR_BUFFER_ERROR when max_chunk is reached); the engine binds the
 * symbol weakly, as libnghttp2 provides it in a real build.
 * Build: gcc -O1 -rdynamic -I include test_compat.c -L<lib> -lnghttp2_amd_hd
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nghttp2_amd_hd_huffman_compat.h"

#define ERR_BUFFER_ERROR (-502)
#define ERR_HEADER_COMP (-523)

static int failures = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);      \
      ++failures;                                                       \
    }                                                                   \
  } while (0)

/* ---- nghttp2_bufs test double (lib/nghttp2_buf.c semantics) ---- */
static nghttp2_buf_chain *chain_new(size_t len) {
  nghttp2_buf_chain *c = calloc(1, sizeof(*c));
  c->buf.begin = c->buf.pos = c->buf.last = c->buf.mark = malloc(len ? len : 1);
  c->buf.end = c->buf.begin + len;
  return c;
}

static void bufs_init(nghttp2_bufs *b, size_t chunk, size_t max_chunk) {
  memset(b, 0, sizeof(*b));
  b->head = b->cur = chain_new(chunk);
  b->chunk_length = chunk;
  b->max_chunk = max_chunk;
  b->chunk_used = 1;
}

static void bufs_free(nghttp2_bufs *b) {
  nghttp2_buf_chain *c = b->head;
  while (c) {
    nghttp2_buf_chain *n = c->next;
    free(c->buf.begin);
    free(c);
    c = n;
  }
}

/* lib/nghttp2_buf.c:294-324 + :372-383 */
int nghttp2_bufs_addb(nghttp2_bufs *bufs, uint8_t b) {
  if (bufs->cur->buf.end == bufs->cur->buf.last) {
    if (bufs->cur->next) {
      bufs->cur = bufs->cur->next;
    } else {
      if (bufs->max_chunk == bufs->chunk_used) return ERR_BUFFER_ERROR;
      bufs->cur->next = chain_new(bufs->chunk_length);
      bufs->cur = bufs->cur->next;
      ++bufs->chunk_used;
    }
  }
  *bufs->cur->buf.last++ = b;
  return 0;
}

static size_t bufs_gather(nghttp2_bufs *b, uint8_t *out) {
  size_t n = 0;
  for (nghttp2_buf_chain *c = b->head; c; c = c->next) {
    size_t k = (size_t)(c->buf.last - c->buf.pos);
    memcpy(out + n, c->buf.pos, k);
    n += k;
  }
  return n;
}

static void buf_wrap(nghttp2_buf *buf, uint8_t *b, size_t len) {
  buf->begin = buf->pos = buf->last = buf->mark = b;
  buf->end = b + len;
}

int main(void) {
  /* test_nghttp2_hd_huff_encode: bytes 22..0 round trip (28/30-bit codes) */
  {
    static const uint8_t t1[] = {22, 21, 20, 19, 18, 17, 16, 15, 14, 13, 12, 11,
                                 10, 9,  8,  7,  6,  5,  4,  3,  2,  1,  0};
    nghttp2_bufs bufs;
    nghttp2_buf outbuf;
    nghttp2_hd_huff_decode_context ctx;
    uint8_t enc[256], b[256];
    bufs_init(&bufs, 4096, 16);
    CHECK(nghttp2_hd_huff_encode(&bufs, t1, sizeof(t1)) == 0);
    size_t elen = bufs_gather(&bufs, enc);
    CHECK(elen == nghttp2_hd_huff_encode_count(t1, sizeof(t1)));
    buf_wrap(&outbuf, b, sizeof(b));
    nghttp2_hd_huff_decode_context_init(&ctx);
    nghttp2_ssize len = nghttp2_hd_huff_decode(&ctx, &outbuf, enc, elen, 1);
    CHECK(len == (nghttp2_ssize)elen);
    CHECK((size_t)(outbuf.last - outbuf.pos) == sizeof(t1));
    CHECK(memcmp(t1, outbuf.pos, sizeof(t1)) == 0);
    bufs_free(&bufs);
  }
  /* test_nghttp2_hd_huff_decode */
  {
    static const uint8_t e[] = {0x1F, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF};
    nghttp2_hd_huff_decode_context ctx;
    nghttp2_buf outbuf;
    uint8_t b[256];
    nghttp2_ssize len;

    buf_wrap(&outbuf, b, sizeof(b));
    nghttp2_hd_huff_decode_context_init(&ctx);
    len = nghttp2_hd_huff_decode(&ctx, &outbuf, e, 1, 1);
    CHECK(len == 1);
    CHECK(memcmp("a", outbuf.pos, 1) == 0);

    buf_wrap(&outbuf, b, sizeof(b));
    nghttp2_hd_huff_decode_context_init(&ctx);
    len = nghttp2_hd_huff_decode(&ctx, &outbuf, e, 2, 1);
    CHECK(len == ERR_HEADER_COMP);

    buf_wrap(&outbuf, b, sizeof(b));
    nghttp2_hd_huff_decode_context_init(&ctx);
    len = nghttp2_hd_huff_decode(&ctx, &outbuf, e, 2, 6);
    CHECK(len == ERR_HEADER_COMP);

    buf_wrap(&outbuf, b, sizeof(b));
    nghttp2_hd_huff_decode_context_init(&ctx);
    len = nghttp2_hd_huff_decode(&ctx, &outbuf, e, 5, 0);
    CHECK(len == 5);
    CHECK(nghttp2_hd_huff_decode_failure_state(&ctx));
  }
  /* RFC 7541 C.4.1, and a chunked (streaming) decode of it */
  {
    static const uint8_t h[] = {0xf1, 0xe3, 0xc2, 0xe5, 0xf2, 0x3a,
                                0x6b, 0xa0, 0xab, 0x90, 0xf4, 0xff};
    const char *s = "www.example.com";
    nghttp2_bufs bufs;
    uint8_t enc[64], b[64];
    bufs_init(&bufs, 64, 1);
    CHECK(nghttp2_hd_huff_encode(&bufs, (const uint8_t *)s, strlen(s)) == 0);
    CHECK(bufs_gather(&bufs, enc) == sizeof(h) && memcmp(enc, h, sizeof(h)) == 0);
    bufs_free(&bufs);
    for (size_t cut = 0; cut <= sizeof(h); ++cut) {
      nghttp2_hd_huff_decode_context ctx;
      nghttp2_buf outbuf;
      buf_wrap(&outbuf, b, sizeof(b));
      nghttp2_hd_huff_decode_context_init(&ctx);
      CHECK(nghttp2_hd_huff_decode(&ctx, &outbuf, h, cut, 0) == (nghttp2_ssize)cut);
      CHECK(nghttp2_hd_huff_decode(&ctx, &outbuf, h + cut, sizeof(h) - cut, 1) ==
            (nghttp2_ssize)(sizeof(h) - cut));
      CHECK((size_t)(outbuf.last - outbuf.pos) == strlen(s));
      CHECK(memcmp(outbuf.pos, s, strlen(s)) == 0);
    }
  }
  /* chain spill: 1000 bytes into 7-byte chunks; then wrap-mode overflow */
  {
    uint8_t raw[1000], enc[4096], b[4096];
    for (int i = 0; i < 1000; ++i) raw[i] = (uint8_t)(i * 37 + 11);
    size_t need = nghttp2_hd_huff_encode_count(raw, sizeof(raw));
    nghttp2_bufs bufs;
    bufs_init(&bufs, 7, 100000);
    CHECK(nghttp2_hd_huff_encode(&bufs, raw, sizeof(raw)) == 0);
    CHECK(bufs_gather(&bufs, enc) == need);
    CHECK(bufs.chunk_used == (need + 6) / 7);
    bufs_free(&bufs);
    nghttp2_hd_huff_decode_context ctx;
    nghttp2_buf outbuf;
    buf_wrap(&outbuf, b, sizeof(b));
    nghttp2_hd_huff_decode_context_init(&ctx);
    CHECK(nghttp2_hd_huff_decode(&ctx, &outbuf, enc, need, 1) == (nghttp2_ssize)need);
    CHECK((size_t)(outbuf.last - outbuf.pos) == sizeof(raw) &&
          memcmp(outbuf.pos, raw, sizeof(raw)) == 0);
    /* one chunk, one byte short: BUFFER_ERROR after filling it */
    bufs_init(&bufs, need - 1, 1);
    CHECK(nghttp2_hd_huff_encode(&bufs, raw, sizeof(raw)) == ERR_BUFFER_ERROR);
    CHECK((size_t)(bufs.head->buf.last - bufs.head->buf.pos) == need - 1);
    CHECK(memcmp(bufs.head->buf.pos, enc, need - 1) == 0);
    bufs_free(&bufs);
  }
  if (failures) {
    fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  printf("compat OK\n");
  return 0;
}
