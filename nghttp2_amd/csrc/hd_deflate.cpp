// hd_deflate.cpp -- batched HPACK deflate front-end (the
// deflate side of rows 1 and 3).
//
// Host C++ above the C ABI.  Deflates many header lists (blocks of one or
// many connections) per call; every string literal of the batch is framed by
// ONE GPU call (nghttp2_amd_hd_emit_strings_batch: Huffman-or-raw choice,
// H bit, length prefix, payload) instead of one emit_string per literal:
//   pass 1  per block in order, against its deflater's dynamic table: table
//           size updates, the table search, the indexing decision and the
//           insertion -- the representation bytes, and the literals to frame;
//   GPU     H2D of the literal strings, emit_strings, D2H of the literals;
//   pass 2  the wire of each block: representation bytes and framed literals
//           in order.
// Output equals nghttp2_hd_deflate_hd2 (nghttp2.h:6127) per block:
// nghttp2_hd_deflate_hd_bufs (lib/nghttp2_hd.c:1469-1505), deflate_nv
// (:1373-1467), search_hd_table / search_static_table / hd_map_find
// (:1201-1249, :566-589), hd_deflate_decide_indexing (:1358-1371),
// emit_indexed_block / emit_indname_block / emit_newname_block /
// emit_table_size (:975-1128), add_hd_table_incremental (:1130-1195).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <deque>
#include <unordered_map>
#include <mutex>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "../../include/nghttp2_amd_hd.h"
#include "../../include/nghttp2_amd_hd_testing.h"
#include "host_threads.h"
#include "hd_tokens.h"

namespace {

const uint32_t kEntryOverhead = 32;
const uint32_t kStaticLen = 61;
const char *const kStatic[kStaticLen][2] = {
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

enum Mode { WITH_INDEXING, WITHOUT_INDEXING, NEVER_INDEXING };  // nghttp2_hd.h

bool name_is(const uint8_t *name, size_t len, const char *s) {
  return strlen(s) == len && memcmp(s, name, len) == 0;
}

// lookup_token (lib/nghttp2_hd.c:137) and name_hash (:536-547): one FNV-1a
// pass and a hashed probe (hd_tokens.h), shared with the GPU kernel.
using hdtok::name_hash;
constexpr int32_t kLastStaticToken = 60;  // NGHTTP2_TOKEN_WWW_AUTHENTICATE

struct Entry {
  std::string name, value;
  uint32_t hash;
};

// RFC 7541 5.1 prefix integer (encode_length, lib/nghttp2_hd.c:840-863)
void put_int(std::string &out, uint32_t n, uint32_t prefix, uint8_t first) {
  const uint32_t k = (1u << prefix) - 1u;
  if (n < k) {
    out.push_back((char)(first | n));
    return;
  }
  out.push_back((char)(first | k));
  n -= k;
  for (; n >= 128u; n >>= 7) out.push_back((char)(0x80u | (n & 0x7Fu)));
  out.push_back((char)n);
}

}  // namespace

struct nghttp2_amd_hd_deflater {
  std::deque<Entry> table;  // front = most recent
  // name hash -> insertion sequence numbers of the entries with that hash,
  // oldest first (the reference's hd_map buckets, lib/nghttp2_hd.c:549-611);
  // the entry with sequence q sits at table[next_seq - 1 - q]
  std::unordered_map<uint32_t, std::deque<uint64_t>> by_hash;
  uint64_t next_seq = 0;
  size_t bufsize = 0;
  size_t bufsize_max;                   // ctx.hd_table_bufsize_max
  size_t deflate_max;                   // deflate_hd_table_bufsize_max
  size_t min_max = UINT32_MAX;          // min_hd_table_bufsize_max
  bool notify = false;                  // notify_table_size_change
  bool bad = false;

  void evict_oldest() {
    const Entry &e = table.back();
    bufsize -= e.name.size() + e.value.size() + kEntryOverhead;
    auto it = by_hash.find(e.hash);
    it->second.pop_front();  // the oldest entry is the oldest of its bucket
    if (it->second.empty()) by_hash.erase(it);
    table.pop_back();
  }
  void shrink() {
    while (bufsize > bufsize_max && !table.empty()) evict_oldest();
  }
  void add(const uint8_t *n, size_t nl, const uint8_t *v, size_t vl, uint32_t h) {
    const size_t room = nl + vl + kEntryOverhead;
    while (bufsize + room > bufsize_max && !table.empty()) evict_oldest();
    if (room > bufsize_max) return;
    table.push_front(Entry{std::string((const char *)n, nl), std::string((const char *)v, vl), h});
    by_hash[h].push_back(next_seq++);
    bufsize += room;
  }
};

namespace {

struct Engine {
  std::mutex mu;
  uint8_t *h_in = nullptr, *h_out = nullptr;
  uint32_t *h_off = nullptr;
  size_t hin_cap = 0, hout_cap = 0, hoff_cap = 0;
  uint8_t *d_in = nullptr, *d_out = nullptr, *d_ws = nullptr;
  uint32_t *d_off = nullptr;
  size_t din_cap = 0, dout_cap = 0, dws_cap = 0, doff_cap = 0;
  uint32_t *h_nt = nullptr, *d_nt = nullptr;  // name tokens and hashes
  size_t hnt_cap = 0, dnt_cap = 0;
};
// Batches of at least this many field names take their tokens and hashes
// from one k_name_tokens launch (NGHTTP2_AMD_GPU_NAMES_MIN; 0 = always);
// smaller ones from the host lookup, which costs less than a GPU round trip.
std::atomic<uint32_t> g_names_min{[] {
  const char *e = getenv("NGHTTP2_AMD_GPU_NAMES_MIN");
  return e ? (uint32_t)strtoul(e, nullptr, 10) : 2048u;
}()};
uint32_t gpu_names_min() { return g_names_min.load(); }
Engine &engine() {
  static Engine e;
  return e;
}
bool hip_ok(hipError_t e, const char *what) {
  if (e == hipSuccess) return true;
  fprintf(stderr, "nghttp2_amd_hd (deflate): %s: %s\n", what, hipGetErrorString(e));
  return false;
}
// Fault injection for the error paths (tests only, like the reference's
// failmalloc suite, tests/failmalloc_test.c): the next n GPU stages of
// nghttp2_amd_hd_deflate_blocks fail before any HIP call.
std::atomic<int> g_fail_gpu{0};
bool fault_inject_gpu() {
  int k = g_fail_gpu.load();
  while (k > 0)
    if (g_fail_gpu.compare_exchange_weak(k, k - 1)) return true;
  return false;
}
bool grow_host(void **p, size_t *cap, size_t need) {
  if (need <= *cap) return true;
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  *cap = 0;
  if (!hip_ok(hipHostMalloc(p, need, hipHostMallocDefault), "hipHostMalloc")) return false;
  *cap = need;
  return true;
}
bool grow_dev(void **p, size_t *cap, size_t need) {
  if (need <= *cap) return true;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  if (!hip_ok(hipMalloc(p, need), "hipMalloc")) return false;
  *cap = need;
  return true;
}

// One piece of a block's wire: representation bytes, then up to two
// literals (indices into the batch's literal list, -1 = none).
struct Piece {
  std::string bytes;
  int32_t lit[2] = {-1, -1};
};

}  // namespace

extern "C" {

// test hooks (include/nghttp2_amd_hd_testing.h)
void nghttp2_amd_hd__test_fail_deflate_gpu(int n) { g_fail_gpu.store(n); }
void nghttp2_amd_hd__set_gpu_names_min(uint32_t n) { g_names_min.store(n); }

int nghttp2_amd_hd_deflate_new(nghttp2_amd_hd_deflater **deflater_ptr,
                               size_t max_deflate_dynamic_table_size) {
  if (!deflater_ptr) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  nghttp2_amd_hd_deflater *d = new (std::nothrow) nghttp2_amd_hd_deflater();
  if (!d) return NGHTTP2_AMD_ERR_NOMEM;
  // nghttp2_hd_deflate_new2 (lib/nghttp2_hd.c:721-748): the table starts at
  // min(4096, max_deflate) and a smaller maximum is announced by a size update
  d->deflate_max = max_deflate_dynamic_table_size;
  d->bufsize_max = 4096;
  if (max_deflate_dynamic_table_size < 4096) {
    d->notify = true;
    d->bufsize_max = max_deflate_dynamic_table_size;
  }
  *deflater_ptr = d;
  return 0;
}

void nghttp2_amd_hd_deflate_del(nghttp2_amd_hd_deflater *deflater) { delete deflater; }

int nghttp2_amd_hd_deflate_change_table_size(nghttp2_amd_hd_deflater *d,
                                             size_t settings_max_dynamic_table_size) {
  if (!d) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  const size_t next = settings_max_dynamic_table_size < d->deflate_max
                          ? settings_max_dynamic_table_size : d->deflate_max;
  d->bufsize_max = next;
  d->min_max = d->min_max < next ? d->min_max : next;
  d->notify = true;
  d->shrink();
  return 0;
}

size_t nghttp2_amd_hd_deflate_get_num_table_entries(nghttp2_amd_hd_deflater *d) {
  return d ? d->table.size() + kStaticLen : 0;
}

int nghttp2_amd_hd_deflate_get_table_entry(nghttp2_amd_hd_deflater *d, size_t idx,
                                           const uint8_t **name, size_t *namelen,
                                           const uint8_t **value, size_t *valuelen) {
  if (!d || idx == 0 || idx > d->table.size() + kStaticLen) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  --idx;
  if (idx < kStaticLen) {
    *name = (const uint8_t *)kStatic[idx][0];
    *namelen = strlen(kStatic[idx][0]);
    *value = (const uint8_t *)kStatic[idx][1];
    *valuelen = strlen(kStatic[idx][1]);
  } else {
    const Entry &e = d->table[idx - kStaticLen];
    *name = (const uint8_t *)e.name.data();
    *namelen = e.name.size();
    *value = (const uint8_t *)e.value.data();
    *valuelen = e.value.size();
  }
  return 0;
}

size_t nghttp2_amd_hd_deflate_get_dynamic_table_size(nghttp2_amd_hd_deflater *d) {
  return d ? d->bufsize : 0;
}

size_t nghttp2_amd_hd_deflate_get_max_dynamic_table_size(nghttp2_amd_hd_deflater *d) {
  return d ? d->bufsize_max : 0;
}

// nghttp2_hd_deflate_bound (lib/nghttp2_hd.c:1596-1621): two size updates of
// at most 6 bytes, per field two 6-byte length prefixes plus the raw bytes.
size_t nghttp2_amd_hd_deflate_bound(nghttp2_amd_hd_deflater *d, const nghttp2_amd_nv *nva,
                                    size_t nvlen) {
  (void)d;
  size_t n = 12 + 12 * nvlen;
  for (size_t i = 0; i < nvlen; ++i) n += nva[i].namelen + nva[i].valuelen;
  return n;
}

int nghttp2_amd_hd_deflate_blocks(nghttp2_amd_hd_deflater *const *deflaters, uint32_t nblocks,
                                  const nghttp2_amd_nv *nva, const uint32_t *block_nv_off,
                                  uint8_t *out, size_t out_cap, uint32_t *out_off,
                                  int32_t *block_status, void *stream) {
  if (nblocks == 0) {
    if (out_off) out_off[0] = 0;
    return 0;
  }
  if (!deflaters || !block_nv_off || !out_off || !block_status || (!nva && block_nv_off[nblocks]))
    return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  for (uint32_t i = 0; i < nblocks; ++i)
    if (!deflaters[i] || block_nv_off[i] > block_nv_off[i + 1]) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;

  using nghttp2_amd_host::parallel_for;
  nghttp2_amd_host::Pool::CallScope scope;  // workers spin between this call's phases only
  nghttp2_amd_host::Phases ph("deflate");
  // ---- the token and hash of every field name of the batch (lookup_token,
  // name_hash; deflate_nv, lib/nghttp2_hd.c:1388-1393): one GPU launch over
  // the batch's names, before any deflater changes (a failure here leaves
  // the deflaters as they were)
  const uint32_t f0 = block_nv_off[0], nf = block_nv_off[nblocks] - f0;
  std::vector<uint32_t> fnt;  // hash[nf], then token[nf]
  if (nf && nf >= gpu_names_min()) {
    std::vector<uint64_t> nbase(nf + 1, 0);
    for (uint32_t k = 0; k < nf; ++k) nbase[k + 1] = nbase[k] + nva[f0 + k].namelen;
    const uint64_t nraw = nbase[nf];
    if (nraw > UINT32_MAX) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
    const size_t in_bytes = ((size_t)nraw + 15u) / 16u * 16u + 16u;
    std::lock_guard<std::mutex> guard(engine().mu);
    Engine &E = engine();
    hipStream_t st = (hipStream_t)stream;
    if (!grow_host((void **)&E.h_in, &E.hin_cap, in_bytes) ||
        !grow_host((void **)&E.h_off, &E.hoff_cap, ((size_t)nf + 1u) * sizeof(uint32_t)) ||
        !grow_host((void **)&E.h_nt, &E.hnt_cap, 2u * (size_t)nf * sizeof(uint32_t)) ||
        !grow_dev((void **)&E.d_in, &E.din_cap, in_bytes) ||
        !grow_dev((void **)&E.d_off, &E.doff_cap, ((size_t)nf + 1u) * sizeof(uint32_t)) ||
        !grow_dev((void **)&E.d_nt, &E.dnt_cap, 2u * (size_t)nf * sizeof(uint32_t)))
      return NGHTTP2_AMD_ERR_NOMEM;
    parallel_for(nf, 4096, [&](size_t k) {
      E.h_off[k] = (uint32_t)nbase[k];
      if (nva[f0 + k].namelen) memcpy(E.h_in + nbase[k], nva[f0 + k].name, nva[f0 + k].namelen);
    });
    E.h_off[nf] = (uint32_t)nraw;
    memset(E.h_in + nraw, 0, in_bytes - nraw);
    if (fault_inject_gpu() ||
        !hip_ok(hipMemcpyAsync(E.d_in, E.h_in, in_bytes, hipMemcpyHostToDevice, st), "H2D") ||
        !hip_ok(hipMemcpyAsync(E.d_off, E.h_off, ((size_t)nf + 1u) * sizeof(uint32_t), hipMemcpyHostToDevice, st), "H2D"))
      return NGHTTP2_AMD_ERR_FATAL;
    int rv = nghttp2_amd_hd_name_tokens_batch(E.d_in, E.d_off, nf, (int32_t *)(E.d_nt + nf), E.d_nt, stream);
    if (rv) return rv;
    if (!hip_ok(hipMemcpyAsync(E.h_nt, E.d_nt, 2u * (size_t)nf * sizeof(uint32_t), hipMemcpyDeviceToHost, st), "D2H") ||
        !hip_ok(hipStreamSynchronize(st), "sync"))
      return NGHTTP2_AMD_ERR_FATAL;
    fnt.assign(E.h_nt, E.h_nt + 2u * (size_t)nf);
    ph.mark("names");
  }
  // ---- pass 1: representations; one task per connection, its lists in
  // batch order (connections are independent)
  std::vector<std::vector<Piece>> pieces(nblocks);
  std::vector<std::vector<std::pair<const uint8_t *, uint32_t>>> blits(nblocks);
  auto deflate_list = [&](uint32_t i) {
    std::vector<std::pair<const uint8_t *, uint32_t>> &L = blits[i];
    auto lit = [&](const uint8_t *p, size_t len) {
      L.emplace_back(p, (uint32_t)len);
      return (int32_t)(L.size() - 1);
    };
      nghttp2_amd_hd_deflater *d = deflaters[i];
    std::vector<Piece> &P = pieces[i];
    if (d->bad) {
      block_status[i] = NGHTTP2_AMD_ERR_HEADER_COMP;
      return;
    }
    block_status[i] = 0;
    if (d->notify) {  // nghttp2_hd_deflate_hd_bufs, lib/nghttp2_hd.c:1477-1494
      const size_t mn = d->min_max;
      d->notify = false;
      d->min_max = UINT32_MAX;
      Piece pc;
      if (d->bufsize_max > mn) put_int(pc.bytes, (uint32_t)mn, 5, 0x20);
      put_int(pc.bytes, (uint32_t)d->bufsize_max, 5, 0x20);
      P.push_back(pc);
    }
    for (uint32_t k = block_nv_off[i]; k < block_nv_off[i + 1]; ++k) {
      const nghttp2_amd_nv &nv = nva[k];
      const uint32_t nh = fnt.empty() ? name_hash(nv.name, nv.namelen) : fnt[k - f0];
      const int32_t token = fnt.empty() ? hdtok::lookup_token(nv.name, nv.namelen, nh)
                                        : (int32_t)fnt[nf + (k - f0)];
      const size_t room = nv.namelen + nv.valuelen + kEntryOverhead;
      // deflate_nv (:1373-1400): never-index authorization, short cookies
      // and fields flagged NO_INDEX; hd_deflate_decide_indexing (:1358-1371)
      Mode mode;
      if (token == 22 /* authorization */ || (token == 31 /* cookie */ && nv.valuelen < 20) ||
          (nv.flags & 1u)) {
        mode = NEVER_INDEXING;
      } else if (token == 3 /* :path */ || token == 20 /* age */ || token == 27 /* content-length */ ||
                 token == 33 /* etag */ || token == 39 /* if-modified-since */ ||
                 token == 40 /* if-none-match */ || token == 45 /* location */ ||
                 token == 54 /* set-cookie */ || room > d->bufsize_max * 3 / 4) {
        mode = WITHOUT_INDEXING;
      } else {
        mode = WITH_INDEXING;
      }
      // search_hd_table (:1225-1249): the dynamic table newest first (an
      // exact match, else the newest name match; name only when never
      // indexing); a static name without a dynamic exact match searches the
      // static table instead
      const bool name_only = mode == NEVER_INDEXING;
      int64_t idx = -1;
      bool exact = false;
      auto bucket = d->by_hash.find(nh);
      if (bucket != d->by_hash.end()) {
        const std::deque<uint64_t> &seqs = bucket->second;
        for (size_t r = seqs.size(); r-- > 0;) {  // newest first
          const size_t t = (size_t)(d->next_seq - 1u - seqs[r]);
          const Entry &e = d->table[t];
          if (e.name.size() != nv.namelen || memcmp(e.name.data(), nv.name, nv.namelen) != 0) continue;
          if (idx < 0) {
            idx = (int64_t)(kStaticLen + t);
            if (name_only) break;
          }
          if (e.value.size() == nv.valuelen && memcmp(e.value.data(), nv.value, nv.valuelen) == 0) {
            idx = (int64_t)(kStaticLen + t);
            exact = true;
            break;
          }
        }
      }
      if (!exact && token >= 0 && token <= kLastStaticToken) {  // search_static_table (:1201-1223)
        idx = token;
        if (!name_only) {
          for (uint32_t s = (uint32_t)token; s < kStaticLen && name_is(nv.name, nv.namelen, kStatic[s][0]); ++s) {
            if (strlen(kStatic[s][1]) == nv.valuelen && memcmp(kStatic[s][1], nv.value, nv.valuelen) == 0) {
              idx = s;
              exact = true;
              break;
            }
          }
        }
      }
      Piece pc;
      if (exact) {  // emit_indexed_block (:975-993)
        put_int(pc.bytes, (uint32_t)idx + 1u, 7, 0x80);
        P.push_back(pc);
        continue;
      }
      if (mode == WITH_INDEXING) d->add(nv.name, nv.namelen, nv.value, nv.valuelen, nh);
      const uint8_t first = mode == WITH_INDEXING ? 0x40 : mode == WITHOUT_INDEXING ? 0x00 : 0x10;
      if (idx < 0) {  // emit_newname_block (:1104-1128)
        pc.bytes.push_back((char)first);
        pc.lit[0] = lit(nv.name, nv.namelen);
      } else {  // emit_indname_block (:1062-1102)
        put_int(pc.bytes, (uint32_t)idx + 1u, mode == WITH_INDEXING ? 6 : 4, first);
      }
      pc.lit[1] = lit(nv.value, nv.valuelen);
      P.push_back(pc);
    }
  };
  {
    // the batch's lists per connection, in batch order; the parallel region
    // only reads `lists` (a vector indexed by connection number)
    std::unordered_map<nghttp2_amd_hd_deflater *, uint32_t> conn_of;
    std::vector<std::vector<uint32_t>> lists;
    for (uint32_t i = 0; i < nblocks; ++i) {
      auto it = conn_of.emplace(deflaters[i], (uint32_t)lists.size()).first;
      if (it->second == lists.size()) lists.emplace_back();
      lists[it->second].push_back(i);
    }
    parallel_for(lists.size(), 1, [&](size_t c) {
      for (uint32_t i : lists[c]) deflate_list(i);
    });
  }
  // literal numbering: block i's literals are litbase[i] + j
  std::vector<uint32_t> litbase(nblocks + 1, 0);
  std::vector<uint64_t> rawbase(nblocks + 1, 0);
  for (uint32_t i = 0; i < nblocks; ++i) {
    uint64_t r = 0;
    for (auto &l : blits[i]) r += l.second;
    litbase[i + 1] = litbase[i] + (uint32_t)blits[i].size();
    rawbase[i + 1] = rawbase[i] + r;
  }

  ph.mark("tables");
  // Pass 1 has changed the deflaters (entries inserted, size updates
  // consumed).  From here on a failure leaves the encoder tables ahead of
  // what the peer will receive, so every deflater of the batch turns bad and
  // every block not failed already reports the error, as
  // nghttp2_hd_deflate_hd_bufs sets ctx.bad on each failure path
  // (lib/nghttp2_hd.c:1509-1516).
  auto fail_batch = [&](int rv) {
    for (uint32_t i = 0; i < nblocks; ++i) {
      deflaters[i]->bad = true;
      if (block_status[i] >= 0) block_status[i] = rv;
      out_off[i + 1] = 0;
    }
    out_off[0] = 0;
    return rv;
  };
  // ---- GPU: frame every literal of the batch (emit_string)
  const uint32_t nl = litbase[nblocks];
  std::lock_guard<std::mutex> guard(engine().mu);
  Engine &E = engine();
  const uint8_t *fr = nullptr;
  const uint32_t *froff = nullptr;
  if (nl) {
    hipStream_t st = (hipStream_t)stream;
    const uint64_t raw = rawbase[nblocks];
    // uint32 offsets: the framed literals (raw + <= 6 prefix bytes each)
    if (nghttp2_amd_hd_emit_strings_bound(raw, nl) > UINT32_MAX)
      return fail_batch(NGHTTP2_AMD_ERR_INVALID_ARGUMENT);
    const size_t in_bytes = ((size_t)raw + 15u) / 16u * 16u + 16u;
    const size_t out_bytes = nghttp2_amd_hd_emit_strings_bound(raw, nl);
    const size_t ws = nghttp2_amd_hd_emit_strings_workspace_size(raw, nl);
    if (!grow_host((void **)&E.h_in, &E.hin_cap, in_bytes) ||
        !grow_host((void **)&E.h_out, &E.hout_cap, out_bytes) ||
        !grow_host((void **)&E.h_off, &E.hoff_cap, 2u * ((size_t)nl + 1u) * sizeof(uint32_t)) ||
        !grow_dev((void **)&E.d_in, &E.din_cap, in_bytes) ||
        !grow_dev((void **)&E.d_out, &E.dout_cap, out_bytes) ||
        !grow_dev((void **)&E.d_ws, &E.dws_cap, ws) ||
        !grow_dev((void **)&E.d_off, &E.doff_cap, 2u * ((size_t)nl + 1u) * sizeof(uint32_t)))
      return fail_batch(NGHTTP2_AMD_ERR_NOMEM);
    // the literal pool and its offsets, block by block
    parallel_for(nblocks, 256, [&](size_t i) {
      uint32_t o = (uint32_t)rawbase[i];
      uint32_t k = litbase[i];
      for (auto &l : blits[i]) {
        E.h_off[k++] = o;
        if (l.second) memcpy(E.h_in + o, l.first, l.second);
        o += l.second;
      }
    });
    E.h_off[nl] = (uint32_t)raw;
    memset(E.h_in + raw, 0, in_bytes - raw);
    uint32_t *d_fo = E.d_off + (nl + 1);
    uint32_t *h_fo = E.h_off + (nl + 1);
    if (fault_inject_gpu() ||
        !hip_ok(hipMemcpyAsync(E.d_in, E.h_in, in_bytes, hipMemcpyHostToDevice, st), "H2D") ||
        !hip_ok(hipMemcpyAsync(E.d_off, E.h_off, (nl + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, st), "H2D"))
      return fail_batch(NGHTTP2_AMD_ERR_FATAL);
    int rv = nghttp2_amd_hd_emit_strings_batch(E.d_in, E.d_off, nl, raw, E.d_out, out_bytes, d_fo,
                                               E.d_ws, ws, stream);
    if (rv) return fail_batch(rv);
    if (!hip_ok(hipMemcpyAsync(h_fo, d_fo, (nl + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, st), "D2H") ||
        !hip_ok(hipStreamSynchronize(st), "sync"))
      return fail_batch(NGHTTP2_AMD_ERR_FATAL);
    if (!hip_ok(hipMemcpyAsync(E.h_out, E.d_out, h_fo[nl], hipMemcpyDeviceToHost, st), "D2H") ||
        !hip_ok(hipStreamSynchronize(st), "sync"))
      return fail_batch(NGHTTP2_AMD_ERR_FATAL);
    fr = E.h_out;
    froff = h_fo;
  }

  ph.mark("gpu");
  // ---- pass 2: each block's wire size, placement in block order, then the
  // bytes (representation bytes and framed literals, in order)
  std::vector<size_t> need(nblocks, 0);
  parallel_for(nblocks, 256, [&](size_t i) {
    size_t n = 0;
    for (const Piece &pc : pieces[i]) {
      n += pc.bytes.size();
      for (int j = 0; j < 2; ++j)
        if (pc.lit[j] >= 0) {
          const uint32_t g = litbase[i] + (uint32_t)pc.lit[j];
          n += froff[g + 1] - froff[g];
        }
    }
    need[i] = n;
  });
  size_t o = 0;
  int ret = 0;
  out_off[0] = 0;
  for (uint32_t i = 0; i < nblocks; ++i) {
    if (block_status[i] == 0 && deflaters[i]->bad) {
      // an earlier block of this deflater ran out of room in this call:
      // later ones fail as nghttp2_hd_deflate_hd_bufs does (:1475-1477)
      block_status[i] = NGHTTP2_AMD_ERR_HEADER_COMP;
    } else if (block_status[i] == 0 && (o + need[i] > out_cap || o + need[i] > UINT32_MAX)) {
      // INSUFF_BUFSIZE in nghttp2_hd_deflate_hd2 (:1546-1547); the deflater turns bad
      block_status[i] = NGHTTP2_AMD_ERR_BUFFER_ERROR;
      deflaters[i]->bad = true;
      ret = NGHTTP2_AMD_ERR_BUFFER_ERROR;
    } else if (block_status[i] == 0) {
      block_status[i] = (int32_t)need[i];
      o += need[i];
    }
    out_off[i + 1] = (uint32_t)o;
  }
  parallel_for(nblocks, 256, [&](size_t i) {
    if (block_status[i] < 0) return;
    uint8_t *w = out + out_off[i];
    for (const Piece &pc : pieces[i]) {
      memcpy(w, pc.bytes.data(), pc.bytes.size());
      w += pc.bytes.size();
      for (int j = 0; j < 2; ++j) {
        if (pc.lit[j] < 0) continue;
        const uint32_t g = litbase[i] + (uint32_t)pc.lit[j];
        const uint32_t a = froff[g], b = froff[g + 1];
        memcpy(w, fr + a, b - a);
        w += b - a;
      }
    }
  });
  ph.mark("wire");
  return ret;
}

ptrdiff_t nghttp2_amd_hd_deflate_hd2(nghttp2_amd_hd_deflater *deflater, uint8_t *buf, size_t buflen,
                                     const nghttp2_amd_nv *nva, size_t nvlen, void *stream) {
  if (!deflater || (!buf && buflen) || (!nva && nvlen) || nvlen > UINT32_MAX)
    return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  const uint32_t nv_off[2] = {0, (uint32_t)nvlen};
  uint32_t out_off[2] = {0, 0};
  int32_t st = 0;
  uint8_t none = 0;
  const int rv = nghttp2_amd_hd_deflate_blocks(&deflater, 1, nva, nv_off, buf ? buf : &none, buflen,
                                               out_off, &st, stream);
  if (st == NGHTTP2_AMD_ERR_BUFFER_ERROR) return NGHTTP2_AMD_ERR_INSUFF_BUFSIZE;  // :1546-1547
  if (st < 0) return st;
  if (rv < 0) return rv;
  return (ptrdiff_t)st;
}

ptrdiff_t nghttp2_amd_hd_deflate_hd_vec2(nghttp2_amd_hd_deflater *deflater, const nghttp2_amd_vec *vec,
                                         size_t veclen, const nghttp2_amd_nv *nva, size_t nvlen,
                                         void *stream) {
  if (!deflater || (!vec && veclen)) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  size_t total = 0;
  for (size_t i = 0; i < veclen; ++i) {
    if (!vec[i].base && vec[i].len) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
    total += vec[i].len;
  }
  // one chunk: the wire straight into it
  if (veclen == 1) return nghttp2_amd_hd_deflate_hd2(deflater, vec[0].base, vec[0].len, nva, nvlen, stream);
  // else the wire into one contiguous scratch buffer, then across the chunks
  // in order (nghttp2_bufs_wrap_init2 fills them one by one).  The scratch is
  // not zero-filled and is capped at the list's bound (an output always fits
  // that, so the cap changes no result).  On INSUFF_BUFSIZE the chunks are
  // left untouched, where the reference leaves the bytes it had written.
  const size_t cap = std::min(total, nghttp2_amd_hd_deflate_bound(deflater, nva, nvlen));
  std::unique_ptr<uint8_t[]> tmp(new (std::nothrow) uint8_t[cap ? cap : 1]);
  if (!tmp) return NGHTTP2_AMD_ERR_NOMEM;
  const ptrdiff_t n = nghttp2_amd_hd_deflate_hd2(deflater, tmp.get(), cap, nva, nvlen, stream);
  if (n < 0) return n;
  size_t o = 0;
  for (size_t i = 0; i < veclen && o < (size_t)n; ++i) {
    const size_t k = std::min(vec[i].len, (size_t)n - o);
    memcpy(vec[i].base, tmp.get() + o, k);
    o += k;
  }
  return n;
}

}  // extern "C"
