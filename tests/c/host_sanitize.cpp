// Host-layer checks under AddressSanitizer + UndefinedBehaviorSanitizer
// (nghttp2_amd/Makefile `asan`; run by tests/test_sanitize.py on the CPU).
//
// Everything here stays on the host: header blocks without Huffman literals
// make no GPU call (nghttp2_amd_hd_inflate_blocks), and neither do header
// lists whose fields all hit the static table (nghttp2_amd_hd_deflate_blocks).
// A fuzzed block that does hold a Huffman literal reaches the GPU decode; with
// no GPU that call fails (NGHTTP2_AMD_ERR_FATAL), which the checks accept --
// the parsing before it is what runs under the sanitizers.
//
//   1. the reference's inflate cases (tests/nghttp2_hd_test.c:577-724, read
//      as data from tests/golden/ref_hd_tests.json) with their expectations;
//   2. randomized malformed blocks (random bytes, representation sequences
//      with over-long and overflowing integers, table size updates, mutated
//      valid blocks) over several inflaters and small output caps, checking
//      every status and record against the buffers;
//   3. static-table-only deflates, inflated back;
//   4. the JSON reader on mutated documents.
//
// Usage: host_sanitize <ref_hd_tests.json> [iterations] [seed]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/nghttp2_amd_hd.h"
#include "../../nghttp2_amd/drivers/json_lite.h"

namespace {

int g_fail = 0;
#define CHECK(c, ...)                                      \
  do {                                                     \
    if (!(c)) {                                            \
      fprintf(stderr, "CHECK failed %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                        \
      fprintf(stderr, "\n");                               \
      ++g_fail;                                            \
    }                                                      \
  } while (0)

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 1) {}
  uint64_t next() {
    s ^= s >> 12;
    s ^= s << 25;
    s ^= s >> 27;
    return s * 2685821657736338717ull;
  }
  uint32_t below(uint32_t n) { return n ? (uint32_t)(next() % n) : 0u; }
};

std::vector<uint8_t> unhex(const std::string &h) {
  std::vector<uint8_t> o;
  for (size_t i = 0; i + 1 < h.size(); i += 2) o.push_back((uint8_t)strtoul(h.substr(i, 2).c_str(), nullptr, 16));
  return o;
}

// RFC 7541 5.1 integer with an n-bit prefix (flags in the first byte)
void put_int(std::vector<uint8_t> &o, uint8_t flags, int n, uint64_t v) {
  const uint64_t m = (1u << n) - 1u;
  if (v < m) {
    o.push_back((uint8_t)(flags | v));
    return;
  }
  o.push_back((uint8_t)(flags | m));
  v -= m;
  while (v >= 128) {
    o.push_back((uint8_t)(0x80 | (v & 0x7F)));
    v >>= 7;
  }
  o.push_back((uint8_t)v);
}

struct Batch {
  std::vector<nghttp2_amd_hd_nv> nva;
  std::vector<uint8_t> arena;
  std::vector<int32_t> status;
  size_t nv_used = 0, ar_used = 0;
  int rv = 0;
};

Batch inflate(const std::vector<nghttp2_amd_hd_inflater *> &inf, const std::vector<std::vector<uint8_t>> &blocks,
              size_t nva_cap, size_t arena_cap) {
  Batch b;
  const uint32_t n = (uint32_t)blocks.size();
  std::vector<const uint8_t *> ptrs(n);
  std::vector<size_t> lens(n);
  for (uint32_t i = 0; i < n; ++i) {
    ptrs[i] = blocks[i].empty() ? nullptr : blocks[i].data();
    lens[i] = blocks[i].size();
  }
  b.nva.resize(nva_cap ? nva_cap : 1);
  b.arena.resize(arena_cap ? arena_cap : 1);
  b.status.assign(n ? n : 1, 12345);
  b.rv = nghttp2_amd_hd_inflate_blocks(inf.data(), n, ptrs.data(), lens.data(), b.nva.data(), nva_cap,
                                       &b.nv_used, b.arena.data(), arena_cap, &b.ar_used, b.status.data(),
                                       nullptr);
  return b;
}

// 1. the reference's inflate cases
void reference_cases(const jl::Value &ref) {
  const jl::Value *cases = ref.get("inflate_cases");
  CHECK(cases && cases->kind == jl::Value::ARR, "inflate_cases missing");
  if (!cases) return;
  int ran = 0;
  for (auto &cp : cases->arr) {
    const jl::Value &c = *cp;
    const std::string test = c.get("test")->s;
    if (test.find("zero_length_huffman") != std::string::npos) continue;  // (a Huffman literal: GPU)
    nghttp2_amd_hd_inflater *inf = nullptr;
    CHECK(nghttp2_amd_hd_inflate_new(&inf) == 0, "inflate_new");
    for (auto &v : c.get("settings")->arr) nghttp2_amd_hd_inflate_change_table_size(inf, (size_t)v->i);
    Batch b = inflate({inf}, {unhex(c.get("block")->s)}, 64, 4096);
    const jl::Value *exp = c.get("expect");
    if (const jl::Value *rv = exp->get("rv")) {
      CHECK(b.status[0] == rv->i, "%s: status %d, expected %lld", test.c_str(), b.status[0], (long long)rv->i);
    } else {
      const auto &want = exp->get("fields")->arr;
      CHECK(b.status[0] == (int32_t)want.size(), "%s: %d fields", test.c_str(), b.status[0]);
      for (size_t k = 0; k < want.size() && k < b.nv_used; ++k) {
        const nghttp2_amd_hd_nv &r = b.nva[k];
        std::string nm((const char *)b.arena.data() + r.name_off, r.name_len);
        std::string vl((const char *)b.arena.data() + r.value_off, r.value_len);
        CHECK(nm == want[k]->arr[0]->s && vl == want[k]->arr[1]->s, "%s: field %zu", test.c_str(), k);
      }
    }
    nghttp2_amd_hd_inflate_del(inf);
    ++ran;
  }
  printf("reference inflate cases: %d\n", ran);
}

// 2. randomized malformed blocks
std::vector<uint8_t> random_block(Rng &r, const std::vector<std::vector<uint8_t>> &seeds) {
  std::vector<uint8_t> o;
  switch (r.below(4)) {
    case 0: {  // random bytes
      const uint32_t n = r.below(48);
      for (uint32_t i = 0; i < n; ++i) o.push_back((uint8_t)r.next());
      break;
    }
    case 1:
    case 2: {  // representation sequences, mostly well formed
      const uint32_t reps = 1 + r.below(8);
      for (uint32_t k = 0; k < reps; ++k) {
        const uint32_t kind = r.below(6);
        auto idx = [&]() -> uint64_t {
          const uint32_t t = r.below(10);
          return t < 6 ? r.below(62) : t < 8 ? 62 + r.below(40) : t < 9 ? r.next() >> r.below(64) : 0;
        };
        auto lit = [&]() {
          const bool huff = r.below(16) == 0;  // (rare: reaches the GPU decode)
          const uint32_t len = r.below(12) == 0 ? 200 + r.below(3000) : r.below(20);
          const uint32_t have = r.below(8) == 0 ? r.below(len + 1) : len;  // sometimes truncated
          put_int(o, huff ? 0x80 : 0x00, 7, r.below(32) == 0 ? (r.next() >> r.below(64)) : len);
          for (uint32_t i = 0; i < have; ++i) o.push_back((uint8_t)(0x20 + r.below(95)));
        };
        if (kind == 0) {
          put_int(o, 0x80, 7, idx());
        } else if (kind == 1 || kind == 2) {  // incremental indexing, new or indexed name
          const uint64_t i = kind == 1 ? 0 : idx();
          put_int(o, 0x40, 6, i);
          if (!i) lit();
          lit();
        } else if (kind == 3) {  // without indexing / never indexed
          const uint64_t i = r.below(2) ? 0 : idx();
          put_int(o, r.below(2) ? 0x10 : 0x00, 4, i);
          if (!i) lit();
          lit();
        } else {  // dynamic table size update
          const uint32_t t = r.below(8);
          put_int(o, 0x20, 5, t < 5 ? r.below(5000) : t < 7 ? (r.next() >> r.below(64)) : 0);
        }
      }
      if (r.below(8) == 0 && !o.empty()) o.resize(r.below((uint32_t)o.size()));  // cut anywhere
      break;
    }
    default: {  // a mutated valid block
      if (seeds.empty()) break;
      o = seeds[r.below((uint32_t)seeds.size())];
      const uint32_t m = 1 + r.below(4);
      for (uint32_t k = 0; k < m && !o.empty(); ++k) {
        const uint32_t at = r.below((uint32_t)o.size());
        switch (r.below(3)) {
          case 0: o[at] ^= (uint8_t)(1u << r.below(8)); break;
          case 1: o.resize(at); break;
          default: o.insert(o.begin() + at, (uint8_t)r.next()); break;
        }
      }
    }
  }
  return o;
}

void fuzz_inflate(const std::vector<std::vector<uint8_t>> &seeds, uint32_t iters, uint64_t seed) {
  Rng r(seed);
  uint64_t blocks = 0, ok = 0, comp = 0, buf = 0, fatal = 0;
  for (uint32_t it = 0; it < iters; ++it) {
    const uint32_t ninf = 1 + r.below(3);
    std::vector<nghttp2_amd_hd_inflater *> pool(ninf);
    for (auto &p : pool) {
      CHECK(nghttp2_amd_hd_inflate_new(&p) == 0, "inflate_new");
      const uint32_t t = r.below(6);
      if (t == 0) nghttp2_amd_hd_inflate_change_table_size(p, 0);
      else if (t == 1) nghttp2_amd_hd_inflate_change_table_size(p, (size_t)-1);  // (saturating bounds)
      else if (t == 2) nghttp2_amd_hd_inflate_change_table_size(p, r.below(8192));
    }
    // several batches on the same inflaters: the sticky bad state and the
    // table evolution carry over
    for (uint32_t rep = 0; rep < 3; ++rep) {
      const uint32_t nb = r.below(9);
      std::vector<std::vector<uint8_t>> bl(nb);
      std::vector<nghttp2_amd_hd_inflater *> inf(nb);
      for (uint32_t i = 0; i < nb; ++i) {
        bl[i] = random_block(r, seeds);
        inf[i] = pool[r.below(ninf)];
      }
      const size_t nva_cap = r.below(4) == 0 ? r.below(6) : 256;
      const size_t arena_cap = r.below(4) == 0 ? r.below(200) : 1u << 16;
      Batch b = inflate(inf, bl, nva_cap, arena_cap);
      CHECK(b.rv == 0 || b.rv == NGHTTP2_AMD_ERR_BUFFER_ERROR || b.rv == NGHTTP2_AMD_ERR_FATAL ||
                b.rv == NGHTTP2_AMD_ERR_NOMEM,
            "inflate_blocks rv %d", b.rv);
      CHECK(b.nv_used <= nva_cap && b.ar_used <= arena_cap, "used %zu/%zu of %zu/%zu", b.nv_used,
            b.ar_used, nva_cap, arena_cap);
      for (size_t k = 0; k < b.nv_used; ++k) {
        const nghttp2_amd_hd_nv &v = b.nva[k];
        CHECK(v.block < nb, "record block %u", v.block);
        CHECK((size_t)v.name_off + v.name_len < b.ar_used + 1 && (size_t)v.value_off + v.value_len < b.ar_used + 1,
              "record %zu outside the arena", k);
        CHECK(v.flags <= 1, "flags %u", v.flags);
      }
      for (uint32_t i = 0; i < nb; ++i) {
        const int32_t s = b.status[i];
        CHECK(s >= 0 || s == NGHTTP2_AMD_ERR_HEADER_COMP || s == NGHTTP2_AMD_ERR_BUFFER_ERROR ||
                  s == NGHTTP2_AMD_ERR_FATAL || s == NGHTTP2_AMD_ERR_NOMEM,
              "block status %d", s);
        ++blocks;
        ok += s >= 0;
        comp += s == NGHTTP2_AMD_ERR_HEADER_COMP;
        buf += s == NGHTTP2_AMD_ERR_BUFFER_ERROR;
        fatal += s == NGHTTP2_AMD_ERR_FATAL;
      }
      for (auto *p : pool) {  // the table accessors on whatever state remains
        const size_t ne = nghttp2_amd_hd_inflate_get_num_table_entries(p);
        for (size_t idx = 1; idx <= ne; idx += 1 + r.below(7)) {
          const uint8_t *nm, *vl;
          size_t nl, vlen;
          if (nghttp2_amd_hd_inflate_get_table_entry(p, idx, &nm, &nl, &vl, &vlen) == 0) {
            volatile uint8_t sink = 0;
            for (size_t x = 0; x < nl; ++x) sink ^= nm[x];
            for (size_t x = 0; x < vlen; ++x) sink ^= vl[x];
            (void)sink;
          }
        }
        (void)nghttp2_amd_hd_inflate_get_dynamic_table_size(p);
      }
    }
    for (auto *p : pool) nghttp2_amd_hd_inflate_del(p);
  }
  printf("fuzzed blocks: %llu (ok %llu, -523 %llu, -502 %llu, fatal %llu)\n", (unsigned long long)blocks,
         (unsigned long long)ok, (unsigned long long)comp, (unsigned long long)buf, (unsigned long long)fatal);
}

// 3. static-table-only deflates, inflated back
void static_deflate(uint32_t iters, uint64_t seed) {
  static const char *kStatic[][2] = {{":method", "GET"},   {":method", "POST"},   {":path", "/"},
                                     {":path", "/index.html"}, {":scheme", "http"}, {":scheme", "https"},
                                     {":status", "200"},   {":status", "204"},    {":status", "206"},
                                     {":status", "304"},   {":status", "400"},    {":status", "404"},
                                     {":status", "500"},   {"accept-encoding", "gzip, deflate"}};
  Rng r(seed);
  for (uint32_t it = 0; it < iters; ++it) {
    const uint32_t nb = 1 + r.below(6);
    std::vector<nghttp2_amd_nv> nva;
    std::vector<uint32_t> off{0};
    for (uint32_t i = 0; i < nb; ++i) {
      const uint32_t k = r.below(8);
      for (uint32_t j = 0; j < k; ++j) {
        const auto &e = kStatic[r.below(14)];
        nva.push_back(nghttp2_amd_nv{(const uint8_t *)e[0], (const uint8_t *)e[1], strlen(e[0]), strlen(e[1]), 0});
      }
      off.push_back((uint32_t)nva.size());
    }
    nghttp2_amd_hd_deflater *d = nullptr;
    CHECK(nghttp2_amd_hd_deflate_new(&d, 4096) == 0, "deflate_new");
    if (r.below(3) == 0) nghttp2_amd_hd_deflate_change_table_size(d, r.below(8192));
    const size_t cap = r.below(5) == 0 ? r.below(8) : 4096;
    std::vector<uint8_t> out(cap ? cap : 1);
    std::vector<uint32_t> out_off(nb + 1);
    std::vector<int32_t> st(nb);
    nghttp2_amd_hd_deflater *ds[8];
    for (uint32_t i = 0; i < nb; ++i) ds[i] = d;
    const int rv = nghttp2_amd_hd_deflate_blocks(ds, nb, nva.data(), off.data(), out.data(), cap, out_off.data(),
                                                 st.data(), nullptr);
    CHECK(rv == 0 || rv == NGHTTP2_AMD_ERR_BUFFER_ERROR, "deflate_blocks rv %d", rv);
    if (rv == 0) {
      nghttp2_amd_hd_inflater *inf = nullptr;
      nghttp2_amd_hd_inflate_new(&inf);
      std::vector<std::vector<uint8_t>> bl(nb);
      std::vector<nghttp2_amd_hd_inflater *> infs(nb, inf);
      for (uint32_t i = 0; i < nb; ++i) {
        CHECK(out_off[i + 1] >= out_off[i] && out_off[i + 1] <= cap, "out_off");
        bl[i].assign(out.begin() + out_off[i], out.begin() + out_off[i + 1]);
      }
      Batch b = inflate(infs, bl, 256, 1 << 16);
      CHECK(b.rv == 0, "inflate back rv %d", b.rv);
      size_t k = 0;
      for (uint32_t i = 0; i < nb; ++i) {
        CHECK(b.status[i] == (int32_t)(off[i + 1] - off[i]), "block %u fields %d", i, b.status[i]);
        for (uint32_t j = off[i]; j < off[i + 1] && k < b.nv_used; ++j, ++k) {
          const auto &r2 = b.nva[k];
          CHECK(r2.name_len == nva[j].namelen && !memcmp(b.arena.data() + r2.name_off, nva[j].name, r2.name_len),
                "name");
          CHECK(r2.value_len == nva[j].valuelen &&
                    !memcmp(b.arena.data() + r2.value_off, nva[j].value, r2.value_len),
                "value");
        }
      }
      nghttp2_amd_hd_inflate_del(inf);
    }
    (void)nghttp2_amd_hd_deflate_bound(d, nva.data(), nva.size());
    nghttp2_amd_hd_deflate_del(d);
  }
  printf("static deflates: %u\n", iters);
}

// 4. the JSON reader on mutated documents
void fuzz_json(const std::string &doc, uint32_t iters, uint64_t seed) {
  Rng r(seed);
  uint32_t parsed = 0;
  for (uint32_t it = 0; it < iters; ++it) {
    // a slice of the document, or (one in four) the whole of it with few edits
    const bool whole = r.below(4) == 0;
    const size_t a = whole ? 0 : r.below((uint32_t)doc.size());
    std::string t = whole ? doc : doc.substr(a, 1 + r.below(4000));
    const uint32_t m = whole ? r.below(3) : r.below(6);
    for (uint32_t k = 0; k < m && !t.empty(); ++k) {
      const size_t at = r.below((uint32_t)t.size());
      static const char kJunk[] = "{}[]\",:\\u00e9-+.eE0123456789truefalsenull \t\n\x01\xff";
      switch (r.below(3)) {
        case 0: t[at] = kJunk[r.below(sizeof(kJunk) - 1)]; break;
        case 1: t.erase(at, 1 + r.below(8)); break;
        default: t.insert(at, 1, kJunk[r.below(sizeof(kJunk) - 1)]); break;
      }
    }
    jl::Reader rd(t);
    jl::Ptr v = rd.parse();
    if (v) {
      ++parsed;
      std::string o;
      jl::dump(o, *v, 0);
    }
  }
  printf("json documents: %u (%u parsed)\n", iters, parsed);
}

}  // namespace

int main(int argc, char **argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s <ref_hd_tests.json> [iterations] [seed]\n", argv[0]);
    return 2;
  }
  const uint32_t iters = argc > 2 ? (uint32_t)atoi(argv[2]) : 2000;
  const uint64_t seed = argc > 3 ? strtoull(argv[3], nullptr, 0) : 1;
  FILE *f = fopen(argv[1], "rb");
  std::string text;
  if (!f || !jl::read_file(f, text)) {
    fprintf(stderr, "cannot read %s\n", argv[1]);
    return 2;
  }
  fclose(f);
  jl::Reader rd(text);
  jl::Ptr ref = rd.parse();
  if (!ref) {
    fprintf(stderr, "bad JSON: %s\n", rd.err().c_str());
    return 2;
  }
  reference_cases(*ref);
  std::vector<std::vector<uint8_t>> seeds;
  for (auto &c : ref->get("inflate_cases")->arr) seeds.push_back(unhex(c->get("block")->s));
  fuzz_inflate(seeds, iters, seed);
  static_deflate(iters / 4 + 1, seed + 7);
  fuzz_json(text, iters, seed + 13);
  if (g_fail) {
    fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  printf("host_sanitize: ok\n");
  return 0;
}
