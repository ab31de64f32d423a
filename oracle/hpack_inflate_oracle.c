/* oracle/hpack_inflate_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A C restatement of nghttp2's HPACK inflater for whole blocks (in_final=1,
 * then end_headers), the same algorithm as oracle/hpack_oracle.py's Inflater,
 * compiled so that the batched inflate front-end (nghttp2_amd_hd_inflate_blocks)
 * has a CPU baseline at C speed (tools/bench_rows.py) beside its parity checker.
 * Huffman literals go through huff_oracle.c (orc_decode, fin=1).  Nothing in the
 * product links it.
 *
 * Restates (citations are /root/reference paths):
 *   nghttp2_hd_inflate_hd_nv              lib/nghttp2_hd.c:1919-2281
 *   nghttp2_hd_inflate_change_table_size  lib/nghttp2_hd.c:1290-1322
 *   decode_length                         lib/nghttp2_hd.c:882-945
 *   hd_inflate_commit_indexed/newname/indname  lib/nghttp2_hd.c:1780-1875
 *   add_hd_table_incremental              lib/nghttp2_hd.c:1130-1195
 *   static table                          RFC 7541 Appendix A
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct { /* as huff_oracle.c */
  uint16_t fstate;
  uint8_t flags;
} orc_ctx;
void orc_decode_context_init(orc_ctx *ctx);
long orc_decode(orc_ctx *ctx, uint8_t *dst, size_t *written, const uint8_t *src, size_t srclen,
                int final);
int orc_decode_failure_state(const orc_ctx *ctx);
int orc_init(void);

#define OHI_MAX_NV 65536u
#define OHI_OVERHEAD 32u
#define OHI_DEFAULT 4096u
#define OHI_HEADER_COMP (-523)

static const char *const kStatic[61][2] = {
    {":authority", ""}, {":method", "GET"}, {":method", "POST"}, {":path", "/"},
    {":path", "/index.html"}, {":scheme", "http"}, {":scheme", "https"}, {":status", "200"},
    {":status", "204"}, {":status", "206"}, {":status", "304"}, {":status", "400"},
    {":status", "404"}, {":status", "500"}, {"accept-charset", ""},
    {"accept-encoding", "gzip, deflate"}, {"accept-language", ""}, {"accept-ranges", ""},
    {"accept", ""}, {"access-control-allow-origin", ""}, {"age", ""}, {"allow", ""},
    {"authorization", ""}, {"cache-control", ""}, {"content-disposition", ""},
    {"content-encoding", ""}, {"content-language", ""}, {"content-length", ""},
    {"content-location", ""}, {"content-range", ""}, {"content-type", ""}, {"cookie", ""},
    {"date", ""}, {"etag", ""}, {"expect", ""}, {"expires", ""}, {"from", ""}, {"host", ""},
    {"if-match", ""}, {"if-modified-since", ""}, {"if-none-match", ""}, {"if-range", ""},
    {"if-unmodified-since", ""}, {"last-modified", ""}, {"link", ""}, {"location", ""},
    {"max-forwards", ""}, {"proxy-authenticate", ""}, {"proxy-authorization", ""},
    {"range", ""}, {"referer", ""}, {"refresh", ""}, {"retry-after", ""}, {"server", ""},
    {"set-cookie", ""}, {"strict-transport-security", ""}, {"transfer-encoding", ""},
    {"user-agent", ""}, {"vary", ""}, {"via", ""}, {"www-authenticate", ""}};

typedef struct {
  uint8_t *nv;  /* name then value, one allocation (like an rcbuf pair) */
  size_t nl, vl;
} ohi_entry;

typedef struct {
  ohi_entry *ring; /* ring[(first + k) % cap]: k = 0 the oldest */
  size_t cap, first, count;
  size_t size, max, settings_max, min_max;
  int expect_size, bad;
} ohi;

ohi *ohi_new(void) {
  if (orc_init()) return NULL; /* the Huffman tables (idempotent) */
  ohi *h = (ohi *)calloc(1, sizeof(ohi));
  if (!h) return NULL;
  h->max = h->settings_max = OHI_DEFAULT;
  h->min_max = 0xFFFFFFFFu;
  return h;
}

void ohi_del(ohi *h) {
  if (!h) return;
  for (size_t k = 0; k < h->count; ++k) free(h->ring[(h->first + k) % h->cap].nv);
  free(h->ring);
  free(h);
}

static void evict_oldest(ohi *h) {
  ohi_entry *e = &h->ring[h->first];
  h->size -= e->nl + e->vl + OHI_OVERHEAD;
  free(e->nv);
  h->first = (h->first + 1) % h->cap;
  --h->count;
}

static void shrink(ohi *h) {
  while (h->size > h->max && h->count) evict_oldest(h);
}

/* lib/nghttp2_hd.c:1290-1322 */
void ohi_change_table_size(ohi *h, size_t v) {
  h->settings_max = v;
  if (h->max > v) {
    h->expect_size = 1;
    h->min_max = v;
    h->max = v;
    shrink(h);
  }
}

/* newest first: k = 0 is dynamic index 62 */
static const ohi_entry *get_dyn(const ohi *h, size_t k) {
  return &h->ring[(h->first + h->count - 1 - k) % h->cap];
}

/* add_hd_table_incremental: copies name and value before evicting */
static int add(ohi *h, const uint8_t *n, size_t nl, const uint8_t *v, size_t vl) {
  const size_t room = nl + vl + OHI_OVERHEAD;
  uint8_t *nv = (uint8_t *)malloc(nl + vl + 1);
  if (!nv) return -1;
  if (nl) memcpy(nv, n, nl);
  if (vl) memcpy(nv + nl, v, vl);
  while (h->size + room > h->max && h->count) evict_oldest(h);
  if (room > h->max) {
    free(nv);
    return 0;
  }
  if (h->count == h->cap) {
    const size_t nc = h->cap ? 2 * h->cap : 16;
    ohi_entry *r = (ohi_entry *)malloc(nc * sizeof(ohi_entry));
    if (!r) {
      free(nv);
      return -1;
    }
    for (size_t k = 0; k < h->count; ++k) r[k] = h->ring[(h->first + k) % h->cap];
    free(h->ring);
    h->ring = r;
    h->cap = nc;
    h->first = 0;
  }
  ohi_entry *e = &h->ring[(h->first + h->count) % h->cap];
  e->nv = nv;
  e->nl = nl;
  e->vl = vl;
  ++h->count;
  h->size += room;
  return 0;
}

size_t ohi_num_entries(const ohi *h) { return h->count; }
size_t ohi_table_size(const ohi *h) { return h->size; }
void ohi_get_entry(const ohi *h, size_t k, const uint8_t **n, size_t *nl, const uint8_t **v, size_t *vl) {
  const ohi_entry *e = get_dyn(h, k);
  *n = e->nv;
  *nl = e->nl;
  *v = e->nv + e->nl;
  *vl = e->vl;
}

typedef struct {
  const uint8_t *b;
  size_t len, pos;
} rd;

/* decode_length (lib/nghttp2_hd.c:882-945) with in_final; -1 on failure */
static int read_int(rd *r, unsigned prefix, uint32_t maxlen, uint32_t *out) {
  if (r->pos >= r->len) return -1;
  const uint32_t k = (1u << prefix) - 1u;
  uint32_t n = r->b[r->pos++] & k;
  if (n == k) {
    for (uint32_t shift = 0;; shift += 7) {
      if (r->pos >= r->len) return -1;
      const uint32_t c = r->b[r->pos++];
      uint32_t a = c & 0x7Fu;
      if (shift >= 32 || (0xFFFFFFFFu >> shift) < a) return -1;
      a <<= shift;
      if (0xFFFFFFFFu - a < n) return -1;
      n += a;
      if (!(c & 0x80u)) break;
    }
  }
  if (n > maxlen) return -1;
  *out = n;
  return 0;
}

/* a string literal: raw bytes in place, or Huffman-decoded into `scratch` */
static int read_str(rd *r, uint8_t *scratch, const uint8_t **s, size_t *sl) {
  if (r->pos >= r->len) return -1;
  const int huff = r->b[r->pos] & 0x80;
  uint32_t n;
  if (read_int(r, 7, OHI_MAX_NV, &n)) return -1;
  if (r->len - r->pos < n) return -1;
  const uint8_t *p = r->b + r->pos;
  r->pos += n;
  if (!huff) {
    *s = p;
    *sl = n;
    return 0;
  }
  orc_ctx ctx;
  orc_decode_context_init(&ctx);
  size_t w = 0;
  const long rv = orc_decode(&ctx, scratch, &w, p, n, 1);
  if (rv < 0 || orc_decode_failure_state(&ctx)) return -1;
  *s = scratch;
  *sl = w;
  return 0;
}

/* emit a field: name\0value\0 into the arena, 5 words into nv */
static int emit(uint8_t *arena, size_t acap, size_t *aused, uint32_t *nv, size_t nvcap, size_t *nvused,
                const uint8_t *n, size_t nl, const uint8_t *v, size_t vl, uint32_t flags) {
  if (*nvused >= nvcap || *aused + nl + vl + 2 > acap) return -2;
  uint32_t *f = nv + 5 * *nvused;
  f[0] = (uint32_t)*aused;
  f[1] = (uint32_t)nl;
  if (nl) memcpy(arena + *aused, n, nl);
  *aused += nl;
  arena[(*aused)++] = 0;
  f[2] = (uint32_t)*aused;
  f[3] = (uint32_t)vl;
  if (vl) memcpy(arena + *aused, v, vl);
  *aused += vl;
  arena[(*aused)++] = 0;
  f[4] = flags;
  ++*nvused;
  return 0;
}

/* One block.  Returns the number of fields, OHI_HEADER_COMP (the fields
 * before the error stay emitted, the inflater turns bad), or -2 when the
 * caller's arena / field buffers are too small. */
long ohi_inflate_block(ohi *h, const uint8_t *b, size_t len, uint8_t *arena, size_t acap,
                       size_t *aused, uint32_t *nv, size_t nvcap, size_t *nvused) {
  *aused = 0;
  *nvused = 0;
  if (h->bad) return OHI_HEADER_COMP;
  static __thread uint8_t sn[OHI_MAX_NV * 8 / 5 + 8], sv[OHI_MAX_NV * 8 / 5 + 8];
  rd r = {b, len, 0};
  int head = 1;
  while (r.pos < r.len) {
    const uint8_t c = r.b[r.pos];
    if (h->expect_size && (c & 0xE0) != 0x20) goto fail;
    if ((c & 0xE0) == 0x20) {
      if (!head) goto fail;
      uint32_t v;
      const size_t lim = h->min_max < h->settings_max ? h->min_max : h->settings_max;
      if (read_int(&r, 5, lim > 0xFFFFFFFFu ? 0xFFFFFFFFu : (uint32_t)lim, &v)) goto fail;
      h->min_max = 0xFFFFFFFFu;
      h->expect_size = 0;
      h->max = v;
      shrink(h);
      continue;
    }
    head = 0;
    const uint32_t maxidx = (uint32_t)(h->count + 61);
    if (c & 0x80) {
      uint32_t idx;
      if (read_int(&r, 7, maxidx, &idx) || idx == 0) goto fail;
      const uint8_t *n, *v;
      size_t nl, vl;
      if (idx - 1 < 61) {
        n = (const uint8_t *)kStatic[idx - 1][0];
        nl = strlen(kStatic[idx - 1][0]);
        v = (const uint8_t *)kStatic[idx - 1][1];
        vl = strlen(kStatic[idx - 1][1]);
      } else {
        ohi_get_entry(h, idx - 1 - 61, &n, &nl, &v, &vl);
      }
      if (emit(arena, acap, aused, nv, nvcap, nvused, n, nl, v, vl, 0)) return -2;
      continue;
    }
    const int index_required = (c & 0x40) != 0;
    const int no_index = (c & 0xF0) == 0x10;
    const uint8_t *n, *v;
    size_t nl, vl;
    if (c == 0x40 || c == 0x00 || c == 0x10) {
      ++r.pos;
      if (read_str(&r, sn, &n, &nl)) goto fail;
    } else {
      uint32_t idx;
      if (read_int(&r, index_required ? 6 : 4, maxidx, &idx) || idx == 0) goto fail;
      if (idx - 1 < 61) {
        n = (const uint8_t *)kStatic[idx - 1][0];
        nl = strlen(kStatic[idx - 1][0]);
      } else {
        const uint8_t *v0;
        size_t vl0;
        ohi_get_entry(h, idx - 1 - 61, &n, &nl, &v0, &vl0);
      }
    }
    if (read_str(&r, sv, &v, &vl)) goto fail;
    /* the field is emitted (copied) before the table insertion may evict
     * the entry its name points into */
    if (emit(arena, acap, aused, nv, nvcap, nvused, n, nl, v, vl, no_index ? 1u : 0u)) return -2;
    if (index_required) {
      const uint32_t *f = nv + 5 * (*nvused - 1);
      if (add(h, arena + f[0], nl, arena + f[2], vl)) return -2;
    }
  }
  if (h->expect_size) goto fail; /* lib/nghttp2_hd.c:2259-2266 */
  return (long)*nvused;
fail:
  h->bad = 1;
  return OHI_HEADER_COMP;
}

/* ---- CPU baseline: a batch of blocks over T threads, one connection per
 * inflater, each thread owning whole connections (blocks of a connection in
 * batch order), fields into per-thread buffers. ---- */
typedef struct {
  ohi **inf;                 /* per connection */
  const uint8_t *const *blocks;
  const size_t *lens;
  const uint32_t *conn;      /* per block */
  uint32_t nblocks, nconn, t, nt;
  long fields;
  int err;
} ohi_job;

static void *ohi_worker(void *arg) {
  ohi_job *j = (ohi_job *)arg;
  size_t acap = 1 << 20, nvcap = 1 << 14, aused, nvused;
  uint8_t *arena = (uint8_t *)malloc(acap);
  uint32_t *nv = (uint32_t *)malloc(nvcap * 5 * sizeof(uint32_t));
  if (!arena || !nv) {
    j->err = 1;
    free(arena);
    free(nv);
    return NULL;
  }
  for (uint32_t i = 0; i < j->nblocks; ++i) {
    if (j->conn[i] % j->nt != j->t) continue;
    for (;;) {
      const long rv = ohi_inflate_block(j->inf[j->conn[i]], j->blocks[i], j->lens[i], arena, acap,
                                        &aused, nv, nvcap, &nvused);
      if (rv != -2) {
        if (rv > 0) j->fields += rv;
        break;
      }
      j->err = 1; /* buffers too small for one block: never for the benchmark's blocks */
      break;
    }
  }
  free(arena);
  free(nv);
  return NULL;
}

/* Inflate the batch with fresh inflaters, nthreads threads; returns the
 * wall seconds (CLOCK_MONOTONIC) and the fields emitted, or < 0 on error. */
double ohi_inflate_batch_timed(const uint8_t *const *blocks, const size_t *lens, const uint32_t *conn,
                               uint32_t nblocks, uint32_t nconn, int nthreads, long *fields) {
  if (orc_init()) return -1.0;
  if (nthreads < 1) nthreads = 1;
  ohi **inf = (ohi **)calloc(nconn, sizeof(ohi *));
  ohi_job *jobs = (ohi_job *)calloc((size_t)nthreads, sizeof(ohi_job));
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  double dt = -1.0;
  if (!inf || !jobs || !th) goto out;
  for (uint32_t c = 0; c < nconn; ++c)
    if (!(inf[c] = ohi_new())) goto out;
  struct timespec a, z;
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (int t = 0; t < nthreads; ++t) {
    jobs[t] = (ohi_job){inf, blocks, lens, conn, nblocks, nconn, (uint32_t)t, (uint32_t)nthreads, 0, 0};
    if (pthread_create(&th[t], NULL, ohi_worker, &jobs[t])) goto out;
  }
  *fields = 0;
  for (int t = 0; t < nthreads; ++t) {
    pthread_join(th[t], NULL);
    *fields += jobs[t].fields;
    if (jobs[t].err) *fields = -1;
  }
  clock_gettime(CLOCK_MONOTONIC, &z);
  dt = (double)(z.tv_sec - a.tv_sec) + 1e-9 * (double)(z.tv_nsec - a.tv_nsec);
out:
  if (inf)
    for (uint32_t c = 0; c < nconn; ++c) ohi_del(inf[c]);
  free(inf);
  free(jobs);
  free(th);
  return dt;
}
