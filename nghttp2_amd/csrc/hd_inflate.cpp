// hd_inflate.cpp -- batched HPACK inflate front-end.
//
// Host C++ above the C ABI.  Inflates many complete header blocks (of one or
// many connections) per call and sends every Huffman literal of the batch
// through ONE GPU decode (nghttp2_amd_hd_huff_decode_batch_auto), instead of
// one nghttp2_hd_huff_decode per literal:
//   pass 1  parse each block's representations and literal extents (the
//           wire is self-delimiting: no table state needed), collecting the
//           Huffman literals into one pinned pool;
//   GPU     H2D, batch decode, D2H (async on the caller's stream);
//   pass 2  replay the blocks in batch order against each inflater's dynamic
//           table -- index resolution, insertion with eviction, table size
//           updates -- and emit the header fields.
// Semantics follow nghttp2_hd_inflate_hd_nv (lib/nghttp2_hd.c:1919-2281) with
// in_final = 1 and nghttp2_hd_inflate_end_headers after each block:
// decode_length (:882-945) with its overflow and maximum checks, the table
// size update rules (:1942-2003, nghttp2_hd_inflate_change_table_size
// :1290-1322), commit_indexed / newname / indname (:1780-1875),
// add_hd_table_incremental (:1130-1195), and the sticky bad state (:1932).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <deque>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/nghttp2_amd_hd.h"

namespace {

const uint32_t kMaxNv = 65536;         // NGHTTP2_HD_MAX_NV
const uint32_t kEntryOverhead = 32;    // NGHTTP2_HD_ENTRY_OVERHEAD
const uint32_t kDefaultTable = 4096;   // NGHTTP2_HD_DEFAULT_MAX_BUFFER_SIZE
const uint32_t kStaticLen = 61;

// RFC 7541 Appendix A
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

struct Entry {
  std::string name, value;
};

}  // namespace

struct nghttp2_amd_hd_inflater {
  std::deque<Entry> table;  // front = most recent (dynamic index 62)
  size_t bufsize = 0;
  size_t bufsize_max = kDefaultTable;           // ctx.hd_table_bufsize_max
  size_t settings_max = kDefaultTable;          // settings_hd_table_bufsize_max
  size_t min_max = UINT32_MAX;                  // min_hd_table_bufsize_max
  bool expect_size = false;                     // NGHTTP2_HD_STATE_EXPECT_TABLE_SIZE
  bool bad = false;                             // ctx.bad

  // Undo log of the block being applied: a block that runs out of caller
  // buffer space is rolled back so the inflater is as before the call.
  std::vector<Entry> evicted;  // in eviction order
  size_t pushed = 0;

  void evict() {
    bufsize -= table.back().name.size() + table.back().value.size() + kEntryOverhead;
    evicted.push_back(std::move(table.back()));
    table.pop_back();
  }
  void shrink() {  // hd_context_shrink_table_size
    while (bufsize > bufsize_max && !table.empty()) evict();
  }
  void add(const std::string &name, const std::string &value) {  // add_hd_table_incremental
    const size_t room = name.size() + value.size() + kEntryOverhead;
    while (bufsize + room > bufsize_max && !table.empty()) evict();
    if (room > bufsize_max) return;
    table.push_front(Entry{name, value});
    bufsize += room;
    ++pushed;
  }
  void begin_block() {
    evicted.clear();
    pushed = 0;
  }
  void rollback() {  // newest entries out, evicted ones back in reverse order
    for (; pushed; --pushed) {
      bufsize -= table.front().name.size() + table.front().value.size() + kEntryOverhead;
      table.pop_front();
    }
    while (!evicted.empty()) {
      bufsize += evicted.back().name.size() + evicted.back().value.size() + kEntryOverhead;
      table.push_back(std::move(evicted.back()));
      evicted.pop_back();
    }
  }
  size_t max_index() const { return table.size() + kStaticLen; }  // get_max_index
};

namespace {

// decode_length (lib/nghttp2_hd.c:882-945) for a whole block: the prefix
// integer at in[*pos]; false on overflow or truncation.
bool read_int(const uint8_t *in, size_t len, size_t *pos, uint32_t prefix, uint32_t *out) {
  if (*pos >= len) return false;
  const uint32_t k = (1u << prefix) - 1u;
  uint32_t n = in[*pos] & k;
  ++*pos;
  if (n != k) {
    *out = n;
    return true;
  }
  for (uint32_t shift = 0;; shift += 7) {
    if (*pos >= len) return false;  // truncated (in_final)
    const uint32_t b = in[(*pos)++];
    uint32_t add = b & 0x7Fu;
    if (shift >= 32) return false;
    if ((UINT32_MAX >> shift) < add) return false;
    add <<= shift;
    if (UINT32_MAX - add < n) return false;
    n += add;
    if (!(b & 0x80u)) break;
  }
  *out = n;
  return true;
}

// A string literal: raw bytes, or a Huffman literal decoded on the GPU.
struct Lit {
  const uint8_t *p;
  uint32_t len;
  int32_t huff;  // index into the batch's Huffman literals, or -1
};
// One representation of a block (parsed in pass 1).
struct Op {
  enum Kind : uint8_t { SIZE, INDEXED, LITERAL } kind;
  bool index_required = false, no_index = false, new_name = false;
  uint32_t value = 0;  // SIZE: the new size; INDEXED / indexed-name LITERAL: the index
  Lit name{nullptr, 0, -1}, val{nullptr, 0, -1};
};
struct Block {
  std::vector<Op> ops;
  bool parse_ok = true;
};

struct Engine {
  std::mutex mu;
  uint8_t *h_pool = nullptr;  // pinned: Huffman literals in, decoded out
  size_t h_cap = 0;
  uint32_t *h_meta = nullptr;  // pinned: offsets in, slots + status out
  size_t m_cap = 0;
  uint8_t *d_in = nullptr, *d_out = nullptr;
  uint32_t *d_off = nullptr, *d_slot = nullptr;
  int32_t *d_st = nullptr;
  size_t din_cap = 0, dout_cap = 0, dn_cap = 0;
};
Engine &engine() {
  static Engine e;
  return e;
}

bool hip_ok(hipError_t e, const char *what) {
  if (e == hipSuccess) return true;
  fprintf(stderr, "nghttp2_amd_hd (inflate): %s: %s\n", what, hipGetErrorString(e));
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

// Pass 1: representations and literal extents of one block
// (lib/nghttp2_hd.c:1942-1985 opcode dispatch; string literal = H bit,
// 7-bit-prefix length <= NGHTTP2_HD_MAX_NV, bytes).
bool parse_block(const uint8_t *in, size_t len, Block &b) {
  size_t pos = 0;
  auto read_lit = [&](Lit &l) {
    if (pos >= len) return false;
    const bool h = in[pos] & 0x80u;
    uint32_t n;
    if (!read_int(in, len, &pos, 7, &n) || n > kMaxNv || len - pos < n) return false;
    l.p = in + pos;
    l.len = n;
    l.huff = h ? 0 : -1;
    pos += n;
    return true;
  };
  b.ops.reserve(len / 4 + 1);
  while (pos < len) {
    Op op;
    const uint8_t c = in[pos];
    if ((c & 0xE0u) == 0x20u) {  // dynamic table size update
      op.kind = Op::SIZE;
      if (!read_int(in, len, &pos, 5, &op.value)) return false;
    } else if (c & 0x80u) {  // indexed
      op.kind = Op::INDEXED;
      if (!read_int(in, len, &pos, 7, &op.value)) return false;
    } else {
      op.kind = Op::LITERAL;
      op.index_required = (c & 0x40u) != 0;
      op.no_index = (c & 0xF0u) == 0x10u;
      if (c == 0x40u || c == 0 || c == 0x10u) {
        op.new_name = true;
        ++pos;
        if (!read_lit(op.name)) return false;
      } else if (!read_int(in, len, &pos, op.index_required ? 6 : 4, &op.value)) {
        return false;
      }
      if (!read_lit(op.val)) return false;
    }
    b.ops.push_back(op);
  }
  return true;
}

// The Huffman literals of a block's parsed representations.
void collect_huff(Block &b, std::vector<Lit *> &huff) {
  for (Op &op : b.ops) {
    if (op.kind != Op::LITERAL) continue;
    if (op.name.huff == 0) huff.push_back(&op.name);
    if (op.val.huff == 0) huff.push_back(&op.val);
  }
}

}  // namespace

extern "C" {

int nghttp2_amd_hd_inflate_new(nghttp2_amd_hd_inflater **inflater_ptr) {
  if (!inflater_ptr) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  *inflater_ptr = new (std::nothrow) nghttp2_amd_hd_inflater();
  return *inflater_ptr ? 0 : NGHTTP2_AMD_ERR_NOMEM;
}

void nghttp2_amd_hd_inflate_del(nghttp2_amd_hd_inflater *inflater) { delete inflater; }

int nghttp2_amd_hd_inflate_change_table_size(nghttp2_amd_hd_inflater *inf,
                                             size_t settings_max_dynamic_table_size) {
  if (!inf) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  inf->settings_max = settings_max_dynamic_table_size;
  if (inf->bufsize_max > settings_max_dynamic_table_size) {
    inf->expect_size = true;
    inf->min_max = settings_max_dynamic_table_size;
    inf->bufsize_max = settings_max_dynamic_table_size;
    inf->shrink();
  }
  return 0;
}

size_t nghttp2_amd_hd_inflate_get_num_table_entries(nghttp2_amd_hd_inflater *inf) {
  return inf ? inf->max_index() : 0;
}

int nghttp2_amd_hd_inflate_get_table_entry(nghttp2_amd_hd_inflater *inf, size_t idx,
                                           const uint8_t **name, size_t *namelen,
                                           const uint8_t **value, size_t *valuelen) {
  if (!inf || idx == 0 || idx > inf->max_index()) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  --idx;
  if (idx < kStaticLen) {
    *name = (const uint8_t *)kStatic[idx][0];
    *namelen = strlen(kStatic[idx][0]);
    *value = (const uint8_t *)kStatic[idx][1];
    *valuelen = strlen(kStatic[idx][1]);
  } else {
    const Entry &e = inf->table[idx - kStaticLen];
    *name = (const uint8_t *)e.name.data();
    *namelen = e.name.size();
    *value = (const uint8_t *)e.value.data();
    *valuelen = e.value.size();
  }
  return 0;
}

size_t nghttp2_amd_hd_inflate_get_dynamic_table_size(nghttp2_amd_hd_inflater *inf) {
  return inf ? inf->bufsize : 0;
}

size_t nghttp2_amd_hd_inflate_get_max_dynamic_table_size(nghttp2_amd_hd_inflater *inf) {
  return inf ? inf->bufsize_max : 0;
}

int nghttp2_amd_hd_inflate_blocks(nghttp2_amd_hd_inflater *const *inflaters, uint32_t nblocks,
                                  const uint8_t *const *blocks, const size_t *block_lens,
                                  nghttp2_amd_hd_nv *nva, size_t nva_cap, size_t *nva_used,
                                  uint8_t *arena, size_t arena_cap, size_t *arena_used,
                                  int32_t *block_status, void *stream) {
  if (nva_used) *nva_used = 0;
  if (arena_used) *arena_used = 0;
  if (nblocks == 0) return 0;
  if (!inflaters || !blocks || !block_lens || !block_status || !nva_used || !arena_used)
    return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  for (uint32_t i = 0; i < nblocks; ++i)
    if (!inflaters[i] || (!blocks[i] && block_lens[i])) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;

  // ---- pass 1
  std::vector<Block> bl(nblocks);
  std::vector<Lit *> huff;
  for (uint32_t i = 0; i < nblocks; ++i) {
    // a malformed block keeps the representations before the error: the
    // reference emits those fields before it fails
    bl[i].parse_ok = parse_block(blocks[i], block_lens[i], bl[i]);
    collect_huff(bl[i], huff);
  }

  // ---- GPU: every Huffman literal of the batch in one decode
  std::lock_guard<std::mutex> guard(engine().mu);
  Engine &E = engine();
  const uint32_t nh = (uint32_t)huff.size();
  std::vector<uint32_t> hoff(nh + 1, 0);
  for (uint32_t k = 0; k < nh; ++k) {
    huff[k]->huff = (int32_t)k;
    hoff[k + 1] = hoff[k] + huff[k]->len;
  }
  const uint8_t *dec = nullptr;
  const uint32_t *slot = nullptr;
  const int32_t *hst = nullptr;
  if (nh) {
    hipStream_t st = (hipStream_t)stream;
    const size_t in_bytes = ((size_t)hoff[nh] + 15u) / 16u * 16u + 16u;
    const size_t out_bytes = nghttp2_amd_hd_huff_decode_bound(hoff[nh], nh);
    const size_t meta = 3u * ((size_t)nh + 1u) * sizeof(uint32_t);
    if (!grow_host((void **)&E.h_pool, &E.h_cap, in_bytes > out_bytes ? in_bytes : out_bytes) ||
        !grow_host((void **)&E.h_meta, &E.m_cap, meta) ||
        !grow_dev((void **)&E.d_in, &E.din_cap, in_bytes) ||
        !grow_dev((void **)&E.d_out, &E.dout_cap, out_bytes) ||
        !grow_dev((void **)&E.d_off, &E.dn_cap, meta))
      return NGHTTP2_AMD_ERR_NOMEM;
    E.d_slot = E.d_off + (nh + 1);
    E.d_st = (int32_t *)(E.d_slot + (nh + 1));
    for (uint32_t k = 0; k < nh; ++k) memcpy(E.h_pool + hoff[k], huff[k]->p, huff[k]->len);
    memset(E.h_pool + hoff[nh], 0, in_bytes - hoff[nh]);
    memcpy(E.h_meta, hoff.data(), (nh + 1) * sizeof(uint32_t));
    if (hipMemcpyAsync(E.d_in, E.h_pool, in_bytes, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(E.d_off, E.h_meta, (nh + 1) * sizeof(uint32_t), hipMemcpyHostToDevice,
                       st) != hipSuccess)
      return NGHTTP2_AMD_ERR_FATAL;
    int rv = nghttp2_amd_hd_huff_decode_batch_auto(E.d_in, E.d_off, nh, E.d_out, out_bytes,
                                                   E.d_slot, E.d_st, nullptr, nullptr, stream);
    if (rv) return rv;
    uint32_t *h_slot = E.h_meta + (nh + 1);
    int32_t *h_st = (int32_t *)(h_slot + (nh + 1));
    if (hipMemcpyAsync(E.h_pool, E.d_out, out_bytes, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(h_slot, E.d_slot, (nh + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost,
                       st) != hipSuccess ||
        hipMemcpyAsync(h_st, E.d_st, nh * sizeof(int32_t), hipMemcpyDeviceToHost, st) !=
            hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return NGHTTP2_AMD_ERR_FATAL;
    dec = E.h_pool;
    slot = h_slot;
    hst = h_st;
  }

  // ---- pass 2: blocks in batch order against their inflaters
  size_t nv_n = 0, ar_n = 0;
  bool full = false;
  auto lit_str = [&](const Lit &l, std::string &out) {
    if (l.huff < 0) {
      out.assign((const char *)l.p, l.len);
      return true;
    }
    const int32_t s = hst[l.huff];
    if (s < 0) return false;  // -523: bad padding or EOS (hd_inflate_read_huff, :1740-1750)
    out.assign((const char *)dec + slot[l.huff], (size_t)s);
    return true;
  };
  auto emit = [&](uint32_t blk, const std::string &name, const std::string &value,
                  uint8_t flags) {
    if (nv_n >= nva_cap || ar_n + name.size() + value.size() + 2 > arena_cap) {
      full = true;
      return;
    }
    nghttp2_amd_hd_nv &o = nva[nv_n++];
    o.block = blk;
    o.flags = flags;
    o.name_off = (uint32_t)ar_n;
    o.name_len = (uint32_t)name.size();
    memcpy(arena + ar_n, name.data(), name.size());
    ar_n += name.size();
    arena[ar_n++] = 0;  // NUL-terminated like the reference's rcbufs (:2112, :2201)
    o.value_off = (uint32_t)ar_n;
    o.value_len = (uint32_t)value.size();
    memcpy(arena + ar_n, value.data(), value.size());
    ar_n += value.size();
    arena[ar_n++] = 0;
  };
  auto get = [&](nghttp2_amd_hd_inflater *inf, uint32_t idx, std::string &n, std::string &v) {
    if (idx < kStaticLen) {
      n = kStatic[idx][0];
      v = kStatic[idx][1];
    } else {
      n = inf->table[idx - kStaticLen].name;
      v = inf->table[idx - kStaticLen].value;
    }
  };
  std::string name, value;
  for (uint32_t i = 0; i < nblocks && !full; ++i) {
    nghttp2_amd_hd_inflater *inf = inflaters[i];
    const size_t nv0 = nv_n, ar0 = ar_n;
    bool ok = !inf->bad;
    bool head = true;  // size updates only at the head of a block
    const size_t sv_max = inf->bufsize_max, sv_min = inf->min_max;
    const bool sv_expect = inf->expect_size;
    inf->begin_block();
    for (size_t k = 0; ok && !full && k < bl[i].ops.size(); ++k) {
      const Op &op = bl[i].ops[k];
      if (inf->expect_size && op.kind != Op::SIZE) {
        ok = false;
        break;
      }
      if (op.kind == Op::SIZE) {
        if (!head || op.value > (inf->min_max < inf->settings_max ? inf->min_max : inf->settings_max)) {
          ok = false;
          break;
        }
        inf->expect_size = false;
        inf->min_max = UINT32_MAX;
        inf->bufsize_max = op.value;
        inf->shrink();
        continue;
      }
      head = false;
      if (op.kind == Op::INDEXED) {  // hd_inflate_commit_indexed
        if (op.value == 0 || op.value > inf->max_index()) {
          ok = false;
          break;
        }
        get(inf, op.value - 1, name, value);
        emit(i, name, value, 0);
        continue;
      }
      if (op.new_name) {  // hd_inflate_commit_newname
        if (!lit_str(op.name, name)) {
          ok = false;
          break;
        }
      } else {  // hd_inflate_commit_indname
        if (op.value == 0 || op.value > inf->max_index()) {
          ok = false;
          break;
        }
        get(inf, op.value - 1, name, value);
      }
      if (!lit_str(op.val, value)) {
        ok = false;
        break;
      }
      if (op.index_required) inf->add(name, value);
      emit(i, name, value, op.no_index ? 1u : 0u);  // NGHTTP2_NV_FLAG_NO_INDEX
    }
    // truncated or malformed wire after the parsed representations; and a
    // block that ends while a table size update is still expected
    // (lib/nghttp2_hd.c:2259-2266)
    if (ok && (!bl[i].parse_ok || inf->expect_size)) ok = false;
    if (full) {
      nv_n = nv0;
      ar_n = ar0;
      inf->rollback();
      inf->bufsize_max = sv_max;
      inf->min_max = sv_min;
      inf->expect_size = sv_expect;
      for (uint32_t j = i; j < nblocks; ++j) block_status[j] = NGHTTP2_AMD_ERR_BUFFER_ERROR;
      break;
    }
    if (!ok) {
      inf->bad = true;  // sticky (lib/nghttp2_hd.c:1932-1934, :2276)
      block_status[i] = NGHTTP2_AMD_ERR_HEADER_COMP;
      // fields emitted before the error stay (the reference emits them one by one)
    } else {
      block_status[i] = (int32_t)(nv_n - nv0);
    }
  }
  *nva_used = nv_n;
  *arena_used = ar_n;
  return full ? NGHTTP2_AMD_ERR_BUFFER_ERROR : 0;
}

}  // extern "C"
