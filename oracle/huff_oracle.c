/*
 * oracle/huff_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of nghttp2's HPACK Huffman codec, used exclusively as the
 * parity checker by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg.  Nothing in the product (nghttp2_amd/, include/) links,
 * loads or calls this file.
 *
 * What it restates (citations are /root/reference paths):
 *   - table construction: mkhufftbl.py:274-397 (tree build, pre-order node
 *     ids with the "all-ones prefix <= 7 bits" accept rule, 4-bit transition
 *     walk, failure sink state 256).  The code lengths are RFC 7541 App. B
 *     data (mkhufftbl.py:15-273); codes are the canonical assignment, which
 *     the pin step proves equal to the reference's table.
 *   - nghttp2_hd_huff_encode_count   lib/nghttp2_hd_huffman.c:34-43
 *   - nghttp2_hd_huff_encode         lib/nghttp2_hd_huffman.c:45-104, over a
 *     single wrap-mode buffer (nghttp2_bufs_wrap_init, lib/nghttp2_buf.c:196)
 *     so overflow reports NGHTTP2_ERR_BUFFER_ERROR (-502) after writing the
 *     same bytes nghttp2_bufs_addb would have written (lib/nghttp2_buf.c:372).
 *   - nghttp2_hd_huff_decode_context_init  lib/nghttp2_hd_huffman.c:106-109
 *   - nghttp2_hd_huff_decode         lib/nghttp2_hd_huffman.c:111-143
 *   - nghttp2_hd_huff_decode_failure_state lib/nghttp2_hd_huffman.c:145-147
 *   - emit_string (Huffman/raw choice, H bit, 7-bit-prefix length)
 *     lib/nghttp2_hd.c:1001-1044, with count_encoded_length / encode_length
 *     lib/nghttp2_hd.c:823-863
 *
 * Parity pinning: oracle/pin_reference.py runs the reference's own table
 * generator (mkhufftbl.py) in the build container and checks these tables
 * byte-for-byte; tests/golden/ holds the reference unit-test vectors
 * (tests/nghttp2_hd_test.c:1605-1670) which tests/test_oracle.py replays.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#include <pthread.h>
#include <time.h>

#define ORC_ERR_BUFFER_ERROR (-502) /* lib/includes/nghttp2/nghttp2.h:282 */
#define ORC_ERR_HEADER_COMP (-523)  /* lib/includes/nghttp2/nghttp2.h:378 */

#define ORC_ACCEPTED 0x01u /* lib/nghttp2_hd_huffman.h:35 */
#define ORC_SYM 0x02u      /* lib/nghttp2_hd_huffman.h:37 */

/* RFC 7541 Appendix B code lengths, symbols 0..256 (256 = EOS). */
static const uint8_t rfc7541_len[257] = {
    13, 23, 28, 28, 28, 28, 28, 28, 28, 24, 30, 28, 28, 30, 28, 28, 28, 28, 28,
    28, 28, 28, 30, 28, 28, 28, 28, 28, 28, 28, 28, 28, 6,  10, 10, 12, 13, 6,
    8,  11, 10, 10, 8,  11, 8,  6,  6,  6,  5,  5,  5,  6,  6,  6,  6,  6,  6,
    6,  7,  8,  15, 6,  12, 10, 13, 6,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,
    7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  8,  7,  8,  13, 19, 13, 14,
    6,  15, 5,  6,  5,  6,  5,  6,  6,  6,  5,  7,  7,  6,  6,  6,  5,  6,  7,
    6,  5,  5,  6,  7,  7,  7,  7,  7,  15, 11, 14, 13, 28, 20, 22, 20, 20, 22,
    22, 22, 23, 22, 23, 23, 23, 23, 23, 24, 23, 24, 24, 22, 23, 24, 23, 23, 23,
    23, 21, 22, 23, 22, 23, 23, 24, 22, 21, 20, 22, 22, 23, 23, 21, 23, 22, 22,
    24, 21, 22, 23, 23, 21, 21, 22, 21, 23, 22, 23, 23, 20, 22, 22, 22, 23, 22,
    22, 23, 26, 26, 20, 19, 22, 23, 22, 25, 26, 26, 26, 27, 27, 26, 24, 25, 19,
    21, 26, 27, 27, 26, 27, 24, 21, 21, 26, 26, 28, 27, 27, 27, 20, 24, 20, 21,
    22, 21, 21, 23, 22, 22, 25, 25, 24, 24, 26, 23, 26, 27, 26, 26, 27, 27, 27,
    27, 27, 28, 27, 27, 27, 27, 27, 26, 30};

typedef struct {
  uint32_t nbits;
  uint32_t code; /* MSB-aligned, as mkhufftbl.py:432 emits it */
} orc_sym;

typedef struct {
  uint16_t fstate;
  uint8_t flags;
  uint8_t sym;
} orc_dec;

typedef struct {
  uint16_t fstate;
  uint8_t flags;
} orc_ctx;

static orc_sym sym_table[257];
static orc_dec dec_table[257][16];
static int tables_ready;

/* ---- tree (mkhufftbl.py:274-312) ---- */
typedef struct onode {
  int term; /* -1 = internal */
  struct onode *child[2];
  int id;
  int accept;
} onode;

static onode pool[1024];
static int pool_used;

static onode *new_node(void) {
  onode *n = &pool[pool_used++];
  n->term = -1;
  n->child[0] = n->child[1] = NULL;
  n->id = -1;
  n->accept = 0;
  return n;
}

static void tree_add(onode *root, int sym, uint32_t code, int nbits) {
  onode *n = root;
  for (int i = nbits - 1; i >= 0; --i) {
    int b = (code >> i) & 1;
    if (!n->child[b]) n->child[b] = new_node();
    n = n->child[b];
  }
  n->term = sym;
}

/* _set_node_id, mkhufftbl.py:314-321: pre-order over internal nodes. */
static int next_id;
static void set_node_id(onode *n, int depth, int all_ones) {
  if (n->term >= 0) return;
  if (depth <= 7 && all_ones) n->accept = 1;
  n->id = next_id++;
  set_node_id(n->child[0], depth + 1, 0);
  set_node_id(n->child[1], depth + 1, all_ones);
}

/* _traverse, mkhufftbl.py:326-350, writing the row of `start` directly in
 * the form _print_transition_table (mkhufftbl.py:358-386) emits. */
static onode *root_node;
static int trans_n;
static void traverse(onode *node, int sym, orc_dec *row, int left) {
  if (left == 0) {
    orc_dec e;
    onode *nd = node;
    if (sym == 256) {
      sym = -1;
      nd = NULL;
    }
    e.flags = 0;
    e.sym = 0;
    if (sym >= 0) {
      e.sym = (uint8_t)sym;
      e.flags |= ORC_SYM;
    }
    if (!nd) {
      e.fstate = 256;
    } else if (nd->term >= 0) {
      e.fstate = 0;
      e.flags |= ORC_ACCEPTED;
    } else {
      e.fstate = (uint16_t)nd->id;
      if (nd->accept) e.flags |= ORC_ACCEPTED;
    }
    row[trans_n++] = e;
    return;
  }
  if (node->term >= 0) node = root_node;
  for (int b = 0; b < 2; ++b) {
    onode *c = node->child[b];
    int nsym = (c->term >= 0) ? c->term : sym;
    traverse(c, nsym, row, left - 1);
  }
}

static void build_rows(onode *n) {
  if (n->term >= 0) return;
  trans_n = 0;
  traverse(n, -1, dec_table[n->id], 4);
  build_rows(n->child[0]);
  build_rows(n->child[1]);
}

int orc_init(void) {
  if (tables_ready) return 0;
  /* canonical code assignment over (length, symbol) order */
  int order[257];
  for (int i = 0; i < 257; ++i) order[i] = i;
  for (int i = 1; i < 257; ++i) { /* insertion sort, stable */
    int v = order[i], j = i - 1;
    while (j >= 0 && rfc7541_len[order[j]] > rfc7541_len[v]) {
      order[j + 1] = order[j];
      --j;
    }
    order[j + 1] = v;
  }
  uint32_t code = 0;
  int prev = rfc7541_len[order[0]];
  pool_used = 0;
  root_node = new_node();
  for (int i = 0; i < 257; ++i) {
    int s = order[i], L = rfc7541_len[s];
    code <<= (L - prev);
    prev = L;
    sym_table[s].nbits = (uint32_t)L;
    sym_table[s].code = code << (32 - L);
    tree_add(root_node, s, code, L);
    ++code;
  }
  next_id = 0;
  set_node_id(root_node, 0, 1);
  if (next_id != 256) return -1;
  build_rows(root_node);
  for (int k = 0; k < 16; ++k) {
    dec_table[256][k].fstate = 256;
    dec_table[256][k].flags = 0;
    dec_table[256][k].sym = 0;
  }
  tables_ready = 1;
  return 0;
}

const void *orc_sym_table(void) { return sym_table; }
const void *orc_dec_table(void) { return dec_table; }

/* ---- lib/nghttp2_hd_huffman.c:34-43 ---- */
size_t orc_encode_count(const uint8_t *src, size_t len) {
  size_t nbits = 0;
  for (size_t i = 0; i < len; ++i) nbits += sym_table[src[i]].nbits;
  return (nbits + 7) / 8;
}

/* ---- lib/nghttp2_hd_huffman.c:45-104, single wrap-mode chunk ----
 * Writes into dst[0..cap).  *outlen receives the bytes written (also on
 * error).  Returns 0 or ORC_ERR_BUFFER_ERROR. */
int orc_encode(uint8_t *dst, size_t cap, const uint8_t *src, size_t srclen,
               size_t *outlen) {
  const uint8_t *end = src + srclen;
  uint64_t code = 0;
  size_t nbits = 0, w = 0;
  size_t avail = cap;
  for (; src != end;) {
    const orc_sym *sym = &sym_table[*src++];
    code |= (uint64_t)sym->code << (32 - nbits);
    nbits += sym->nbits;
    if (nbits < 32) continue;
    if (avail >= 4) {
      uint32_t x = (uint32_t)(code >> 32);
      dst[w] = (uint8_t)(x >> 24);
      dst[w + 1] = (uint8_t)(x >> 16);
      dst[w + 2] = (uint8_t)(x >> 8);
      dst[w + 3] = (uint8_t)x;
      w += 4;
      avail -= 4;
      code <<= 32;
      nbits -= 32;
      continue;
    }
    for (; nbits >= 8;) {
      if (w >= cap) {
        *outlen = w;
        return ORC_ERR_BUFFER_ERROR;
      }
      dst[w++] = (uint8_t)(code >> 56);
      code <<= 8;
      nbits -= 8;
    }
    avail = cap - w;
  }
  for (; nbits >= 8;) {
    if (w >= cap) {
      *outlen = w;
      return ORC_ERR_BUFFER_ERROR;
    }
    dst[w++] = (uint8_t)(code >> 56);
    code <<= 8;
    nbits -= 8;
  }
  if (nbits) {
    if (w >= cap) {
      *outlen = w;
      return ORC_ERR_BUFFER_ERROR;
    }
    dst[w++] = (uint8_t)((uint8_t)(code >> 56) | ((1 << (8 - nbits)) - 1));
  }
  *outlen = w;
  return 0;
}

/* ---- lib/nghttp2_hd_huffman.c:106-109 ---- */
void orc_decode_context_init(orc_ctx *ctx) {
  ctx->fstate = 0;
  ctx->flags = ORC_ACCEPTED;
}

/* ---- lib/nghttp2_hd_huffman.c:111-143 ----
 * dst must hold floor(8*srclen/5) bytes; *written receives bytes written. */
long orc_decode(orc_ctx *ctx, uint8_t *dst, size_t *written,
                const uint8_t *src, size_t srclen, int final) {
  const uint8_t *end = src + srclen;
  orc_dec t;
  size_t w = 0;
  t.fstate = ctx->fstate;
  t.flags = ctx->flags;
  t.sym = 0;
  for (; src != end;) {
    uint8_t c = *src++;
    t = dec_table[t.fstate][c >> 4];
    if (t.flags & ORC_SYM) dst[w++] = t.sym;
    t = dec_table[t.fstate][c & 0xF];
    if (t.flags & ORC_SYM) dst[w++] = t.sym;
  }
  ctx->fstate = t.fstate;
  ctx->flags = t.flags;
  *written = w;
  if (final && !(ctx->flags & ORC_ACCEPTED)) return ORC_ERR_HEADER_COMP;
  return (long)srclen;
}

/* ---- lib/nghttp2_hd_huffman.c:145-147 ---- */
int orc_decode_failure_state(const orc_ctx *ctx) {
  return ctx->fstate == 0x100;
}

/* ------------------------------------------------------------------
 * Batched wrappers (SoA layout identical to the product C-ABI, see
 * include/nghttp2_amd_hd.h).  Threads split the batch into contiguous,
 * byte-balanced shards.
 * ------------------------------------------------------------------ */
typedef struct {
  int kind; /* 0 count, 1 encode, 2 decode */
  const uint8_t *src;
  const uint32_t *src_off;
  uint32_t lo, hi;
  uint32_t *enc_len;        /* count: per-string encoded length */
  const uint32_t *dst_off;  /* encode/decode: output slots */
  uint8_t *dst;
  int32_t *status;          /* decode: len or -523; encode: 0/-502 */
  uint16_t *fstate;         /* decode: optional final ctx */
  uint8_t *flags;
} orc_job;

static void *orc_worker(void *arg) {
  orc_job *j = (orc_job *)arg;
  for (uint32_t i = j->lo; i < j->hi; ++i) {
    const uint8_t *s = j->src + j->src_off[i];
    size_t len = j->src_off[i + 1] - j->src_off[i];
    if (j->kind == 0) {
      j->enc_len[i] = (uint32_t)orc_encode_count(s, len);
    } else if (j->kind == 1) {
      size_t cap = j->dst_off[i + 1] - j->dst_off[i], outlen = 0;
      int rv = orc_encode(j->dst + j->dst_off[i], cap, s, len, &outlen);
      if (j->status) j->status[i] = rv;
    } else {
      orc_ctx ctx;
      size_t w = 0;
      orc_decode_context_init(&ctx);
      long rv = orc_decode(&ctx, j->dst + j->dst_off[i], &w, s, len, 1);
      j->status[i] = rv < 0 ? (int32_t)rv : (int32_t)w;
      if (j->fstate) j->fstate[i] = ctx.fstate;
      if (j->flags) j->flags[i] = ctx.flags;
    }
  }
  return NULL;
}

static int orc_run(orc_job *proto, uint32_t n, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  if ((uint32_t)nthreads > n) nthreads = n ? (int)n : 1;
  orc_job jobs[256];
  pthread_t th[256];
  const uint64_t total = proto->src_off[n] - proto->src_off[0];
  uint32_t lo = 0;
  for (int t = 0; t < nthreads; ++t) {
    uint32_t hi;
    if (t == nthreads - 1) {
      hi = n;
    } else { /* byte-balanced split: first i with off[i] >= target */
      uint64_t target = proto->src_off[0] + total * (uint64_t)(t + 1) / nthreads;
      uint32_t a = lo, b = n;
      while (a < b) {
        uint32_t m = a + (b - a) / 2;
        if (proto->src_off[m] < target) a = m + 1; else b = m;
      }
      hi = a;
    }
    jobs[t] = *proto;
    jobs[t].lo = lo;
    jobs[t].hi = hi;
    lo = hi;
  }
  if (nthreads == 1) {
    orc_worker(&jobs[0]);
    return 0;
  }
  for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, orc_worker, &jobs[t]);
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  return 0;
}

int orc_encode_count_batch(const uint8_t *src, const uint32_t *src_off,
                           uint32_t n, uint32_t *enc_len, int nthreads) {
  orc_job p;
  memset(&p, 0, sizeof(p));
  p.kind = 0; p.src = src; p.src_off = src_off; p.enc_len = enc_len;
  return orc_run(&p, n, nthreads);
}

int orc_encode_batch(const uint8_t *src, const uint32_t *src_off, uint32_t n,
                     const uint32_t *dst_off, uint8_t *dst, int32_t *status,
                     int nthreads) {
  orc_job p;
  memset(&p, 0, sizeof(p));
  p.kind = 1; p.src = src; p.src_off = src_off; p.dst_off = dst_off;
  p.dst = dst; p.status = status;
  return orc_run(&p, n, nthreads);
}

int orc_decode_batch(const uint8_t *src, const uint32_t *src_off, uint32_t n,
                     const uint32_t *dst_off, uint8_t *dst, int32_t *status,
                     uint16_t *fstate, uint8_t *flags, int nthreads) {
  orc_job p;
  memset(&p, 0, sizeof(p));
  p.kind = 2; p.src = src; p.src_off = src_off; p.dst_off = dst_off;
  p.dst = dst; p.status = status; p.fstate = fstate; p.flags = flags;
  return orc_run(&p, n, nthreads);
}

/* Round trip the way the CPU baseline times it: count +
 * encode (emit_string order, lib/nghttp2_hd.c:1009/:1037), then decode with
 * final=1 + failure_state.  Returns elapsed seconds of the two phases. */
static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int orc_roundtrip_timed(const uint8_t *src, const uint32_t *src_off,
                        uint32_t n, uint32_t *enc_off, uint8_t *enc,
                        const uint32_t *dec_off, uint8_t *dec, int32_t *status,
                        int nthreads, double *t_enc, double *t_dec) {
  double t0 = now_s();
  orc_encode_count_batch(src, src_off, n, enc_off + 1, nthreads);
  enc_off[0] = 0;
  for (uint32_t i = 0; i < n; ++i) enc_off[i + 1] += enc_off[i];
  orc_encode_batch(src, src_off, n, enc_off, enc, NULL, nthreads);
  double t1 = now_s();
  orc_decode_batch(enc, enc_off, n, dec_off, dec, status, NULL, NULL, nthreads);
  double t2 = now_s();
  *t_enc = t1 - t0;
  *t_dec = t2 - t1;
  return 0;
}

/* ------------------------------------------------------------------
 * HPACK string literal framing.
 * ------------------------------------------------------------------ */

/* count_encoded_length, lib/nghttp2_hd.c:823-838 */
size_t orc_count_encoded_length(size_t n, size_t prefix) {
  size_t k = ((size_t)1 << prefix) - 1;
  size_t len = 0;
  if (n < k) return 1;
  n -= k;
  ++len;
  for (; n >= 128; n >>= 7, ++len)
    ;
  return len + 1;
}

/* encode_length, lib/nghttp2_hd.c:840-863: the prefix integer of RFC 7541
 * 5.1 into buf, keeping the bits of buf[0] above the prefix. */
size_t orc_encode_length(uint8_t *buf, size_t n, size_t prefix) {
  size_t k = ((size_t)1 << prefix) - 1;
  uint8_t *begin = buf;
  *buf = (uint8_t)(*buf & ~k);
  if (n < k) {
    *buf = (uint8_t)(*buf | n);
    return 1;
  }
  *buf = (uint8_t)(*buf | k);
  ++buf;
  n -= k;
  for (; n >= 128; n >>= 7) *buf++ = (uint8_t)((1 << 7) | (n & 0x7F));
  *buf++ = (uint8_t)n;
  return (size_t)(buf - begin);
}

/* emit_string, lib/nghttp2_hd.c:1001-1044, into one flat buffer: the
 * Huffman form iff nghttp2_hd_huff_encode_count(str) < len, the H bit
 * (0x80) and the 7-bit-prefix length, then the payload.  Returns the bytes
 * written (dst must hold orc_count_encoded_length(len, 7) + len). */
size_t orc_emit_string(uint8_t *dst, const uint8_t *str, size_t len) {
  size_t enclen = orc_encode_count(str, len);
  int huffman = 0;
  if (enclen < len) {
    huffman = 1;
  } else {
    enclen = len;
  }
  const size_t blocklen = orc_count_encoded_length(enclen, 7);
  dst[0] = huffman ? 1 << 7 : 0;
  orc_encode_length(dst, enclen, 7);
  if (huffman) {
    size_t w = 0;
    orc_encode(dst + blocklen, enclen, str, len, &w);
  } else if (len) {
    memcpy(dst + blocklen, str, len);
  }
  return blocklen + enclen;
}

/* Batch: dst_off[n+1] (OUT) and the literals back to back. */
int orc_emit_strings_batch(const uint8_t *src, const uint32_t *src_off, uint32_t n,
                           uint8_t *dst, uint32_t *dst_off) {
  uint64_t o = 0;
  for (uint32_t i = 0; i < n; ++i) {
    dst_off[i] = (uint32_t)o;
    o += orc_emit_string(dst + o, src + src_off[i], src_off[i + 1] - src_off[i]);
  }
  dst_off[n] = (uint32_t)o;
  return 0;
}
