/* test_sharded.c -- the multi-device engine (nghttp2_amd_hd_sharded_*) from
 * C, on the one GPU of the box with the device list repeating device 0:
 * 1, 2 and 3 shards (worker threads, streams, device contexts), host-resident
 * and device-resident variants, against the unsharded oracle result
 * (oracle/huff_oracle.c: the C restatement of lib/nghttp2_hd_huffman.c,
 * linked as the checker only).  Prints "sharded OK" on success. */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nghttp2_amd_hd.h"

/* the oracle (oracle/_build/libhuff_oracle.so) */
typedef struct {
  uint16_t fstate;
  uint8_t flags;
} orc_ctx;
int orc_init(void);
int orc_encode(uint8_t *dst, size_t cap, const uint8_t *src, size_t srclen, size_t *outlen);
void orc_decode_context_init(orc_ctx *ctx);
long orc_decode(orc_ctx *ctx, uint8_t *dst, size_t *written, const uint8_t *src, size_t srclen, int final);

#define CHECK(c, ...)                                              \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);         \
      fprintf(stderr, __VA_ARGS__);                                \
      fprintf(stderr, "\n");                                       \
      exit(1);                                                     \
    }                                                              \
  } while (0)

static uint64_t rng = 0x5EED5EEDull;
static uint32_t rnd(void) {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (uint32_t)(rng >> 11);
}

typedef struct {
  uint8_t *pool;
  uint32_t *off;
  uint32_t n;
} batch;

/* header-like values: lengths 0..400, printable bytes, some control bytes */
static batch gen_raw(uint32_t n) {
  batch b;
  b.n = n;
  b.off = malloc(4u * (n + 1));
  b.off[0] = 0;
  for (uint32_t i = 0; i < n; ++i) b.off[i + 1] = b.off[i] + (rnd() % 8 == 0 ? rnd() % 401 : rnd() % 60);
  b.pool = calloc(b.off[n] + 64, 1);
  for (uint32_t k = 0; k < b.off[n]; ++k) b.pool[k] = rnd() % 50 == 0 ? (uint8_t)rnd() : (uint8_t)(32 + rnd() % 95);
  return b;
}

/* the oracle's unsharded encode of the whole batch */
static batch oracle_encode(const batch *r) {
  batch e;
  e.n = r->n;
  e.off = malloc(4u * (r->n + 1));
  e.pool = calloc((size_t)r->off[r->n] * 4 + 64, 1);
  e.off[0] = 0;
  for (uint32_t i = 0; i < r->n; ++i) {
    size_t w = 0;
    CHECK(orc_encode(e.pool + e.off[i], (size_t)r->off[r->n] * 4 - e.off[i], r->pool + r->off[i],
                     r->off[i + 1] - r->off[i], &w) == 0, "oracle encode");
    e.off[i + 1] = e.off[i] + (uint32_t)w;
  }
  return e;
}

/* encoded strings with random damage (EOS, bad padding, random bytes) */
static void damage(batch *e) {
  for (uint32_t i = 0; i < e->n; i += 7) {
    const uint32_t a = e->off[i], len = e->off[i + 1] - a;
    if (!len) continue;
    if (i % 3 == 0) e->pool[a + rnd() % len] = 0xFF;
    else e->pool[a + len - 1] ^= (uint8_t)(1u << (rnd() % 8));
  }
}

/* status and bytes of every string against the oracle's decode */
static void check_decode(const batch *e, const uint8_t *d, const uint32_t *doff, const int32_t *st,
                         const char *tag) {
  uint8_t *buf = malloc(8u * 70000 / 5 + 16);
  for (uint32_t i = 0; i < e->n; ++i) {
    orc_ctx ctx;
    orc_decode_context_init(&ctx);
    size_t w = 0;
    const long rv = orc_decode(&ctx, buf, &w, e->pool + e->off[i], e->off[i + 1] - e->off[i], 1);
    const int32_t want = rv < 0 ? (int32_t)rv : (int32_t)w;
    CHECK(st[i] == want, "%s: string %u status %d, oracle %d", tag, i, st[i], want);
    CHECK(memcmp(d + doff[i], buf, w) == 0, "%s: string %u bytes", tag, i);
  }
  free(buf);
}

/* the device of each shard: device 0 repeated, or (several GPUs) distinct
 * devices, which exercises the per-thread hipSetDevice, the per-device
 * persistent-grid cache and per-device workspaces and streams */
static int g_devs[4] = {0, 0, 0, 0};

static void host_variant(uint32_t nshards, const batch *r, const batch *e, const batch *bad) {
  int *devs = g_devs;
  nghttp2_amd_hd_sharded *s = NULL;
  CHECK(nghttp2_amd_hd_sharded_new(&s, devs, nshards) == 0, "sharded_new");
  CHECK(nghttp2_amd_hd_sharded_count(s) == nshards, "count");
  char tag[64];
  /* encode == the oracle's unsharded encode, byte for byte and offset for offset */
  const size_t ecap = nghttp2_amd_hd_huff_encode_bound(r->off[r->n], r->n);
  uint8_t *enc = malloc(ecap);
  uint32_t *eoff = malloc(4u * (r->n + 1));
  CHECK(nghttp2_amd_hd_sharded_encode(s, r->pool, r->off, r->n, enc, ecap, eoff) == 0, "sharded_encode");
  CHECK(memcmp(eoff, e->off, 4u * (r->n + 1)) == 0, "%u shards: encoded offsets", nshards);
  CHECK(memcmp(enc, e->pool, e->off[e->n]) == 0, "%u shards: encoded bytes", nshards);
  /* a pool 1 byte short: BUFFER_ERROR, the overflow mark, nothing written */
  memset(enc, 0xAB, ecap);
  CHECK(nghttp2_amd_hd_sharded_encode(s, r->pool, r->off, r->n, enc, e->off[e->n] - 1, eoff) ==
            NGHTTP2_AMD_ERR_BUFFER_ERROR, "short pool");
  CHECK(eoff[r->n] == NGHTTP2_AMD_OFF_OVERFLOW, "overflow mark");
  for (size_t k = 0; k < ecap; ++k) CHECK(enc[k] == 0xAB, "byte %zu written on overflow", k);
  /* decode of valid and of damaged strings == the oracle's, per string */
  for (int v = 0; v < 2; ++v) {
    const batch *x = v ? bad : e;
    const size_t dcap = nghttp2_amd_hd_huff_decode_bound(x->off[x->n], x->n) + 32u * nshards;
    uint8_t *d = malloc(dcap);
    uint32_t *doff = malloc(4u * (x->n + 1));
    int32_t *st = malloc(4u * x->n);
    uint16_t *fs = malloc(2u * x->n);
    uint8_t *fl = malloc(x->n);
    CHECK(nghttp2_amd_hd_sharded_decode(s, x->pool, x->off, x->n, d, dcap, doff, st, fs, fl) == 0,
          "sharded_decode");
    snprintf(tag, sizeof tag, "%u shards, %s", nshards, v ? "damaged" : "valid");
    check_decode(x, d, doff, st, tag);
    for (uint32_t i = 0; i < x->n; ++i) {
      CHECK(doff[i] <= doff[i + 1] || st[i] < 0, "%s: offsets ascend", tag);
      CHECK(st[i] < 0 || doff[i] + (uint32_t)st[i] <= doff[x->n], "%s: inside the pool", tag);
    }
    free(d), free(doff), free(st), free(fs), free(fl);
  }
  free(enc), free(eoff);
  nghttp2_amd_hd_sharded_del(s);
}

/* device-resident: the caller cuts, each shard's buffers on "its" device */
static void dev_variant(uint32_t nshards, const batch *r, const batch *e) {
  int *devs = g_devs;
  nghttp2_amd_hd_sharded *s = NULL;
  CHECK(nghttp2_amd_hd_sharded_new(&s, devs, nshards) == 0, "sharded_new");
  uint32_t cuts[5];
  CHECK(nghttp2_amd_hd_shard_bounds(r->off, r->n, nshards, cuts) == 0, "shard_bounds");
  CHECK(cuts[0] == 0 && cuts[nshards] == r->n, "bounds cover the batch");
  nghttp2_amd_hd_shard sh[4], dh[4];
  memset(sh, 0, sizeof sh);
  memset(dh, 0, sizeof dh);
  for (uint32_t k = 0; k < nshards; ++k) {
    const uint32_t s0 = cuts[k], s1 = cuts[k + 1], n = s1 - s0;
    const uint32_t a = r->off[s0], b = r->off[s1];
    uint32_t *o = malloc(4u * (n + 1));
    for (uint32_t i = 0; i <= n; ++i) o[i] = r->off[s0 + i] - a;  /* rebased */
    void *src, *soff, *dst, *doff;
    const size_t cap = nghttp2_amd_hd_huff_encode_bound(b - a, n);
    CHECK(hipSetDevice(devs[k]) == hipSuccess, "hipSetDevice");
    CHECK(hipMalloc(&src, (b - a) + 64) == hipSuccess && hipMalloc(&soff, 4u * (n + 1)) == hipSuccess &&
              hipMalloc(&dst, cap) == hipSuccess && hipMalloc(&doff, 4u * (n + 1)) == hipSuccess, "hipMalloc");
    CHECK(hipMemcpy(src, r->pool + a, (b - a) + 32, hipMemcpyHostToDevice) == hipSuccess, "H2D");
    CHECK(hipMemcpy(soff, o, 4u * (n + 1), hipMemcpyHostToDevice) == hipSuccess, "H2D");
    sh[k].src = src, sh[k].src_off = soff, sh[k].n = n, sh[k].in_bytes = b - a;
    sh[k].dst = dst, sh[k].dst_cap = cap, sh[k].dst_off = doff;
    free(o);
  }
  CHECK(nghttp2_amd_hd_sharded_encode_dev(s, sh) == 0, "encode_dev");
  for (uint32_t k = 0; k < nshards; ++k) {
    const uint32_t s0 = cuts[k], n = cuts[k + 1] - s0;
    CHECK(sh[k].rv == 0, "shard rv");
    CHECK(sh[k].out_base == e->off[s0], "%u shards: shard %u base %llu, oracle %u", nshards, k,
          (unsigned long long)sh[k].out_base, e->off[s0]);
    CHECK(sh[k].out_bytes == e->off[cuts[k + 1]] - e->off[s0], "shard bytes");
    uint8_t *out = malloc(sh[k].out_bytes + 1);
    uint32_t *oo = malloc(4u * (n + 1));
    CHECK(hipSetDevice(devs[k]) == hipSuccess, "hipSetDevice");
    CHECK(hipMemcpy(out, sh[k].dst, sh[k].out_bytes, hipMemcpyDeviceToHost) == hipSuccess, "D2H");
    CHECK(hipMemcpy(oo, sh[k].dst_off, 4u * (n + 1), hipMemcpyDeviceToHost) == hipSuccess, "D2H");
    for (uint32_t i = 0; i <= n; ++i) CHECK(oo[i] + sh[k].out_base == e->off[s0 + i], "dev offsets");
    CHECK(memcmp(out, e->pool + e->off[s0], sh[k].out_bytes) == 0, "dev encoded bytes");
    /* decode that shard's encoded output where it lies */
    void *d, *doff, *st;
    const size_t dcap = nghttp2_amd_hd_huff_decode_bound(sh[k].out_bytes, n);
    CHECK(hipMalloc(&d, dcap) == hipSuccess && hipMalloc(&doff, 4u * (n + 1)) == hipSuccess &&
              hipMalloc(&st, 4u * (n + 1)) == hipSuccess, "hipMalloc");
    dh[k].src = sh[k].dst, dh[k].src_off = sh[k].dst_off, dh[k].n = n, dh[k].in_bytes = sh[k].out_bytes;
    dh[k].dst = d, dh[k].dst_cap = dcap, dh[k].dst_off = doff, dh[k].status = st;
    free(out), free(oo);
  }
  CHECK(nghttp2_amd_hd_sharded_decode_dev(s, dh) == 0, "decode_dev");
  for (uint32_t k = 0; k < nshards; ++k) {
    const uint32_t s0 = cuts[k], n = cuts[k + 1] - s0;
    uint8_t *d = malloc(dh[k].out_bytes + 1);
    uint32_t *doff = malloc(4u * (n + 1));
    int32_t *st = malloc(4u * (n + 1));
    CHECK(hipSetDevice(devs[k]) == hipSuccess, "hipSetDevice");
    CHECK(hipMemcpy(d, dh[k].dst, dh[k].out_bytes, hipMemcpyDeviceToHost) == hipSuccess, "D2H");
    CHECK(hipMemcpy(doff, dh[k].dst_off, 4u * (n + 1), hipMemcpyDeviceToHost) == hipSuccess, "D2H");
    CHECK(hipMemcpy(st, dh[k].status, 4u * n + 4, hipMemcpyDeviceToHost) == hipSuccess, "D2H");
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t len = r->off[s0 + i + 1] - r->off[s0 + i];
      CHECK(st[i] == (int32_t)len, "dev decode status");
      CHECK(memcmp(d + doff[i], r->pool + r->off[s0 + i], len) == 0, "dev decode bytes");
    }
    (void)hipFree((void *)sh[k].src), (void)hipFree((void *)sh[k].src_off), (void)hipFree(sh[k].dst),
        (void)hipFree(sh[k].dst_off);
    (void)hipFree(dh[k].dst), (void)hipFree(dh[k].dst_off), (void)hipFree(dh[k].status);
    free(d), free(doff), free(st);
  }
  CHECK(hipSetDevice(0) == hipSuccess, "hipSetDevice");
  nghttp2_amd_hd_sharded_del(s);
}

int main(void) {
  CHECK(orc_init() == 0, "oracle init");
  uint32_t cuts[4];
  const uint32_t off0[4] = {0, 0, 0, 0};
  CHECK(nghttp2_amd_hd_shard_bounds(off0, 3, 3, cuts) == 0 && cuts[3] == 3, "bounds of empties");
  const uint32_t desc[3] = {0, 5, 4};
  CHECK(nghttp2_amd_hd_shard_bounds(desc, 2, 2, cuts) == NGHTTP2_AMD_ERR_INVALID_ARGUMENT, "descending");
  batch r = gen_raw(20000), e = oracle_encode(&r), bad = oracle_encode(&r);
  damage(&bad);
  for (uint32_t m = 1; m <= 3; ++m) {
    host_variant(m, &r, &e, &bad);
    dev_variant(m, &r, &e);
  }
  /* more shards than strings */
  batch r3 = gen_raw(2), e3 = oracle_encode(&r3);
  host_variant(3, &r3, &e3, &e3);
  /* several GPUs: the same checks with distinct devices per shard */
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) == hipSuccess && ndev > 1) {
    for (int k = 0; k < 4; ++k) g_devs[k] = k % ndev;
    for (uint32_t m = 2; m <= 4; ++m) {
      host_variant(m, &r, &e, &bad);
      dev_variant(m, &r, &e);
    }
    printf("sharded OK on %d devices\n", ndev < 4 ? ndev : 4);
  }
  printf("sharded OK\n");
  return 0;
}
