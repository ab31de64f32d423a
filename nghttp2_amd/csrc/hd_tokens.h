// hd_tokens.h -- header-name tokens and the FNV-1a name hash.
//
// The reference maps a header name to a token with a generated switch on
// (length, last byte) and a memcmp (lookup_token, lib/nghttp2_hd.c:137-520):
// a static-table name gives the index of its FIRST static entry
// (NGHTTP2_TOKEN_* 0..60, lib/nghttp2_hd.h:57-108), seven more names get
// 61..67 (:109-115), anything else -1.  The deflater hashes a name with
// 32-bit FNV-1a (name_hash, lib/nghttp2_hd.c:536-547; the static table holds
// the same values precomputed, :62-126) before searching its dynamic table.
//
// Here both are one computation: FNV-1a of the name, then a probe of a
// 128-slot open-addressed table keyed by the hash, verified by length and
// bytes.  The table is built at compile time and shared by the host
// (deflater, single-name C ABI) and the GPU kernel (k_name_tokens, staged in
// LDS).  Plain C++17, no HIP: included by .cpp and .hip sources alike.
#ifndef NGHTTP2_AMD_HD_TOKENS_H
#define NGHTTP2_AMD_HD_TOKENS_H

#include <stddef.h>
#include <stdint.h>

namespace hdtok {

constexpr uint32_t kFnvBasis = 2166136261u;
constexpr uint32_t kFnvPrime = 16777619u;  // 1 + 2 + 16 + 128 + 256 + 2^24: the reference's shift-add form
constexpr uint32_t kSlots = 128;            // power of two, > 2 x the 59 names
constexpr uint32_t kNameBytes = 1024;  // names at 4-byte aligned offsets, zero padded

struct TokenName {
  const char *name;
  int32_t token;
};

// lookup_token's names and results (lib/nghttp2_hd.c:137-520).
constexpr TokenName kTokens[] = {
    {":authority", 0}, {":method", 1}, {":path", 3}, {":scheme", 5}, {":status", 7},
    {"accept-charset", 14}, {"accept-encoding", 15}, {"accept-language", 16},
    {"accept-ranges", 17}, {"accept", 18}, {"access-control-allow-origin", 19}, {"age", 20},
    {"allow", 21}, {"authorization", 22}, {"cache-control", 23}, {"content-disposition", 24},
    {"content-encoding", 25}, {"content-language", 26}, {"content-length", 27},
    {"content-location", 28}, {"content-range", 29}, {"content-type", 30}, {"cookie", 31},
    {"date", 32}, {"etag", 33}, {"expect", 34}, {"expires", 35}, {"from", 36}, {"host", 37},
    {"if-match", 38}, {"if-modified-since", 39}, {"if-none-match", 40}, {"if-range", 41},
    {"if-unmodified-since", 42}, {"last-modified", 43}, {"link", 44}, {"location", 45},
    {"max-forwards", 46}, {"proxy-authenticate", 47}, {"proxy-authorization", 48}, {"range", 49},
    {"referer", 50}, {"refresh", 51}, {"retry-after", 52}, {"server", 53}, {"set-cookie", 54},
    {"strict-transport-security", 55}, {"transfer-encoding", 56}, {"user-agent", 57},
    {"vary", 58}, {"via", 59}, {"www-authenticate", 60}, {"te", 61}, {"connection", 62},
    {"keep-alive", 63}, {"proxy-connection", 64}, {"upgrade", 65}, {":protocol", 66},
    {"priority", 67}};
constexpr uint32_t kNumTokens = sizeof(kTokens) / sizeof(kTokens[0]);

constexpr uint32_t cstr_len(const char *s) {
  uint32_t n = 0;
  while (s[n]) ++n;
  return n;
}
constexpr uint32_t fnv1a(const char *s, uint32_t n) {
  uint32_t h = kFnvBasis;
  for (uint32_t i = 0; i < n; ++i) {
    h ^= (uint8_t)s[i];
    h *= kFnvPrime;
  }
  return h;
}

// slot s: hash[s]; meta[s] = 0 (empty) or (token + 1) | len << 8 | name_off << 16
struct Table {
  uint32_t hash[kSlots];
  uint32_t meta[kSlots];
  uint8_t names[kNameBytes];
};

constexpr uint32_t meta_token(uint32_t m) { return (m & 0xFFu) - 1u; }
constexpr uint32_t meta_len(uint32_t m) { return (m >> 8) & 0xFFu; }
constexpr uint32_t meta_off(uint32_t m) { return m >> 16; }

constexpr Table make_table() {
  Table t{};
  uint32_t at = 0;
  for (uint32_t k = 0; k < kNumTokens; ++k) {
    const char *s = kTokens[k].name;
    const uint32_t n = cstr_len(s), h = fnv1a(s, n);
    for (uint32_t i = 0; i < n; ++i) t.names[at + i] = (uint8_t)s[i];
    uint32_t slot = h & (kSlots - 1u);
    while (t.meta[slot]) slot = (slot + 1u) & (kSlots - 1u);
    t.hash[slot] = h;
    t.meta[slot] = (uint32_t)(kTokens[k].token + 1) | (n << 8) | (at << 16);
    at += (n + 3u) & ~3u;
  }
  return t;
}

constexpr Table kTable = make_table();

constexpr uint32_t total_name_bytes() {
  uint32_t at = 0;
  for (uint32_t k = 0; k < kNumTokens; ++k) at += (cstr_len(kTokens[k].name) + 3u) & ~3u;
  return at;
}
static_assert(total_name_bytes() <= kNameBytes, "token names overflow the table");
static_assert(fnv1a("via", 3) == 1762798611u, "FNV-1a differs from the reference's static hash");

// Host lookup: the same probe the kernel runs.
inline uint32_t name_hash(const uint8_t *p, size_t n) {
  uint32_t h = kFnvBasis;
  for (size_t i = 0; i < n; ++i) {
    h ^= p[i];
    h *= kFnvPrime;
  }
  return h;
}
inline int32_t lookup_token(const uint8_t *p, size_t n, uint32_t h) {
  for (uint32_t slot = h & (kSlots - 1u);; slot = (slot + 1u) & (kSlots - 1u)) {
    const uint32_t m = kTable.meta[slot];
    if (m == 0) return -1;
    if (kTable.hash[slot] != h || meta_len(m) != n) continue;
    const uint8_t *q = kTable.names + meta_off(m);
    size_t i = 0;
    while (i < n && q[i] == p[i]) ++i;
    if (i == n) return (int32_t)meta_token(m);
  }
}

}  // namespace hdtok

#endif
