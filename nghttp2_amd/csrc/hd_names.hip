// hd_names.hip -- batched header-name tokenisation and FNV-1a name hash
//  for gfx950.
//
// Reference: lookup_token (lib/nghttp2_hd.c:137-520) and name_hash
// (:536-547), called once per header field by deflate_nv (:1388-1393) and by
// the inflater (:1811).  Here a batch of N names in SoA form (byte pool +
// uint32 offsets[N+1], the Huffman batch layout) gives token[N] (int32,
// lookup_token's result: -1 or NGHTTP2_TOKEN_*) and hash[N] (FNV-1a of the
// name, which equals static_table[token].hash for a static name).
//
// Layout and bound: one lane per name.  FNV-1a is a serial chain per name, so
// each lane walks its own name in 32-byte chunks of aligned 16-byte loads
// (the next chunk in flight while the current one is hashed, branch-free
// predicated steps); the 64 names of a wave are contiguous in the pool, so
// their loads share cache lines and HBM sees each byte once.  The 128-slot
// token table (hd_tokens.h) is staged in LDS once per workgroup (1.6 KB);
// a hash + length hit is verified with dword compares against the name's
// bytes still in registers.  HBM traffic per
// name: its bytes + 4 (offset) in, 8 out -- an HBM-bound byte scan, no MFMA.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/nghttp2_amd_hd.h"
#include "hd_tokens.h"

namespace {

typedef __attribute__((address_space(3))) uint32_t lds_u32;

constexpr uint32_t NT_WG = 256;

__constant__ hdtok::Table kTokTable = hdtok::kTable;

// FNV-1a steps over the bytes [a, b) of the 32-byte chunk at cb (branch-free)
__device__ __forceinline__ uint32_t hash_chunk(uint32_t h, uint4 c0, uint4 c1, uint32_t cb, uint32_t a,
                                               uint32_t b) {
  const uint32_t w[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
  // chunk-relative byte range [lo, hi): each step compares its constant j
  const int32_t lo = (int32_t)(a - cb), hi = (int32_t)(b - cb);
#pragma unroll
  for (int32_t j = 0; j < 32; ++j) {
    const uint32_t c = (w[j >> 2] >> (8u * (j & 3))) & 0xFFu;
    const uint32_t hn = (h ^ c) * hdtok::kFnvPrime;
    h = (j >= lo && j < hi) ? hn : h;
  }
  return h;
}

__global__ __launch_bounds__(NT_WG) void k_name_tokens(const uint8_t *__restrict__ names,
                                                       const uint32_t *__restrict__ off, uint32_t n,
                                                       int32_t *__restrict__ token,
                                                       uint32_t *__restrict__ hash) {
  __shared__ uint32_t th[hdtok::kSlots], tm[hdtok::kSlots];
  __shared__ uint32_t tn[hdtok::kNameBytes / 4];
  for (uint32_t i = threadIdx.x; i < hdtok::kSlots; i += NT_WG) {
    th[i] = kTokTable.hash[i];
    tm[i] = kTokTable.meta[i];
  }
  for (uint32_t i = threadIdx.x; i < hdtok::kNameBytes / 4; i += NT_WG)
    tn[i] = reinterpret_cast<const uint32_t *>(kTokTable.names)[i];
  __syncthreads();  // the only workgroup barrier
  const lds_u32 *TH = (const lds_u32 *)th, *TM = (const lds_u32 *)tm, *TN = (const lds_u32 *)tn;
  const uint32_t s = blockIdx.x * NT_WG + threadIdx.x;
  if (s >= n) return;
  const uint32_t a = off[s], b = off[s + 1], len = b - a;
  // FNV-1a over 32-byte chunks from the 16-byte aligned base below the name,
  // the next chunk's loads issued before the current chunk is hashed.  The
  // first two chunks stay in registers (F) for the token compare: a name of
  // <= 32 bytes lies within them ((a & 15) + 32 <= 47).
  const uint4 *g = reinterpret_cast<const uint4 *>(names);
  uint32_t h = hdtok::kFnvBasis;
  uint32_t cb = a & ~15u;
  uint4 c0 = make_uint4(0, 0, 0, 0), c1 = c0, n0 = c0, n1 = c0;
  if (a < b) {
    c0 = g[cb >> 4];
    c1 = g[(cb >> 4) + 1u];
  }
  if (cb + 32u < b) {
    n0 = g[(cb >> 4) + 2u];
    n1 = g[(cb >> 4) + 3u];
  }
  const uint32_t F[16] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w,
                          n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w};
  h = hash_chunk(h, c0, c1, cb, a, b);
  cb += 32u;
  c0 = n0;
  c1 = n1;
  for (; cb < b; cb += 32u) {
    if (cb + 32u < b) {
      n0 = g[(cb >> 4) + 2u];
      n1 = g[(cb >> 4) + 3u];
    }
    h = hash_chunk(h, c0, c1, cb, a, b);
    c0 = n0;
    c1 = n1;
  }
  // token: probe by hash, verify length and bytes (the name's dwords
  // realigned from F with v_alignbyte; table names are dword aligned and
  // zero padded)
  int32_t tok = -1;
  if (len <= 32u) {
    const uint32_t qw = (a & 15u) >> 2, sh = a & 3u;
    uint32_t G[9];
#pragma unroll
    for (uint32_t j = 0; j < 9u; ++j)
      G[j] = qw == 0 ? F[j] : qw == 1 ? F[j + 1] : qw == 2 ? F[j + 2] : F[j + 3];
    uint32_t nm[8];
#pragma unroll
    for (uint32_t i = 0; i < 8u; ++i) {
      uint32_t v = __builtin_amdgcn_alignbyte(G[i + 1], G[i], sh);
      const uint32_t left = len > 4u * i ? len - 4u * i : 0u;
      nm[i] = left >= 4u ? v : v & ((1u << (8u * left)) - 1u);
    }
    for (uint32_t slot = h & (hdtok::kSlots - 1u), k = 0; k < hdtok::kSlots;
         ++k, slot = (slot + 1u) & (hdtok::kSlots - 1u)) {
      const uint32_t m = TM[slot];
      if (m == 0) break;
      if (TH[slot] != h || hdtok::meta_len(m) != len) continue;
      const lds_u32 *q = TN + (hdtok::meta_off(m) >> 2);
      bool eq = true;
#pragma unroll
      for (uint32_t i = 0; i < 8u; ++i)
        if (4u * i < len) eq = eq && nm[i] == q[i];
      if (eq) {
        tok = (int32_t)hdtok::meta_token(m);
        break;
      }
    }
  }
  token[s] = tok;
  hash[s] = h;
}

}  // namespace

extern "C" {

int nghttp2_amd_hd_name_tokens_batch(const uint8_t *names, const uint32_t *name_off, uint32_t n,
                                     int32_t *token, uint32_t *hash, void *stream) {
  if (n == 0) return 0;
  if (!names || !name_off || !token || !hash) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(k_name_tokens, dim3((n + NT_WG - 1u) / NT_WG), dim3(NT_WG), 0,
                     (hipStream_t)stream, names, name_off, n, token, hash);
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess) return 0;
  fprintf(stderr, "nghttp2_amd_hd: HIP error %s\n", hipGetErrorString(e));
  return NGHTTP2_AMD_ERR_FATAL;
}

int32_t nghttp2_amd_hd_lookup_token(const uint8_t *name, size_t namelen) {
  if (!name && namelen) return -1;
  return hdtok::lookup_token(name, namelen, hdtok::name_hash(name, namelen));
}

uint32_t nghttp2_amd_hd_name_hash(const uint8_t *name, size_t namelen) {
  if (!name) return hdtok::kFnvBasis;
  return hdtok::name_hash(name, namelen);
}

}  // extern "C"
