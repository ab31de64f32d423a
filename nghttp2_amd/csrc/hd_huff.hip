// hd_huff.hip -- MI355X (gfx950) HPACK Huffman engine: kernels + C ABI.
//
// Replaces the reference's scalar loops in lib/nghttp2_hd_huffman.c
// (encode_count :34-43, encode :45-104, decode :111-143) for batches of
// independent header strings laid out SoA in HBM (see
// include/nghttp2_amd_hd.h and DESIGN.md).  Integer/table work only (no
// MFMA): HBM-bound streaming with the code tables staged in LDS.
//
// Kernels
//   k_enc_count     aligned 16-byte chunks of a wave's 64 strings, one per
//                   lane: code bits per string from in-chunk prefixes (LDS)
//                   and a wave scan; per-256-string tile sums
//   k_encode        tile offsets from the tile sums, then bit packing: each
//                   string's EOS-prefix padding (lib/nghttp2_hd_huffman.c:
//                   95-101) counted as length of its last byte, codes combined
//                   into pairs and quads in registers and OR'ed into an LDS
//                   image that leaves as whole big-endian dwords
//   k_decode_items  decode_batch_auto: persistent waves, tasks of 64 strings
//                   (a workgroup range's last ones as 32-string units,
//                   claimed largest first when a wave frees up),
//                   rounds of up to 64 items (a whole string, or a 40-byte
//                   piece of a long one, warmed up and verified; the
//                   64-byte instance cuts a round at an input-byte budget);
//                   a 13-bit two-symbol lookup in LDS read through a
//                   register window over the round's staged words, codes
//                   past 13 bits by one read of a leading-ones table;
//                   symbols through a per-lane LDS region, stored with
//                   unaligned 16-byte stores back to back per task; the
//                   final {fstate, flags} of the
//                   reference's nibble FSM (lib/nghttp2_hd_huffman.c:122-136)
//                   rebuilt exactly from the undecoded tail bits (DESIGN.md
//                   "decode state")
//   k_decode        caller slots (decode_batch), capacity-checked
//   k_decode_fsm    the reference's nibble FSM itself (257x16 table in LDS),
//                   kept as the exact cross-check path and for chunked calls
//   k_slot_len / k_scan_tiles / k_scan_apply   tight decode slots
//                   (floor(8E/5)+1 each)
//   k_enc_count<true> / k_encode<true>   HPACK string literals (emit_string,
//                   lib/nghttp2_hd.c:1001-1044) packed straight into wire
//                   order: prefix (H bit, 7-bit-prefix length) + Huffman or
//                   raw payload
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <atomic>
#include <type_traits>

#include "../../include/nghttp2_amd_hd.h"
#include "../../include/nghttp2_amd_hd_testing.h"

namespace dev {
#define HD_TBL static __device__
#include "hd_huff_tables.inc"
#undef HD_TBL
}  // namespace dev

namespace host {
#define HD_TBL static
#include "hd_huff_tables.inc"
#undef HD_TBL
}  // namespace host

#define WG 256          // lanes per workgroup; also strings per scan tile
#define SCAN_WG 1024
#define DEC_WG_PER_CU 8 // persistent decode grid: 256 CUs x 8 workgroups
#define NUM_CU 256

// Bounds-checked debug build (HD_BOUNDS=1; built beside the product as
// lib/libnghttp2_amd_hd_bounds.so, run by tests/test_bounds_gpu.py): every
// LDS staging, region and image index and every per-string global index the
// hot-path kernels compute is checked against its buffer, and a violation
// records its site in this translation unit's g_hd_bounds (one word per
// lane, plain vector stores; nghttp2_amd_hd__bounds_check reports the first
// nonzero word and clears them).  In the product (0) the checks compile to
// nothing.
#ifndef HD_BOUNDS
#define HD_BOUNDS 0
#endif
#if HD_BOUNDS
static __device__ uint32_t g_hd_bounds[64];
#define HD_CHECK(ok, site)                                              \
  do {                                                                  \
    if (!(ok)) g_hd_bounds[threadIdx.x & 63u] = (uint32_t)(site);       \
  } while (0)
#define HD_LIM(x) , (x)
#else
#define HD_CHECK(ok, site) \
  do {                     \
  } while (0)
#define HD_LIM(x)
#endif

#define HUFF_ACCEPTED 0x01u
#define HUFF_SYM 0x02u
#define FAIL_STATE 0x100u

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
// Wave-wide inclusive scans on DPP (row shifts within 16-lane rows, then
// row broadcasts of lanes 15 and 31): VALU only, no LDS round trips.
// Lanes whose DPP source lies outside the row read 0, the identity of
// add / max / or over unsigned values.
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint32_t dpp0(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, false);
}
#define WAVE_SCAN(v, OP)                                                        \
  do {                                                                          \
    v = OP(v, dpp0<0x111>(v));                                                  \
    v = OP(v, dpp0<0x112>(v));                                                  \
    v = OP(v, dpp0<0x114>(v));                                                  \
    v = OP(v, dpp0<0x118>(v));                                                  \
    v = OP(v, dpp0<0x142, 0xa>(v));                                             \
    v = OP(v, dpp0<0x143, 0xc>(v));                                             \
  } while (0)
__device__ __forceinline__ uint32_t op_add(uint32_t a, uint32_t b) { return a + b; }
__device__ __forceinline__ uint32_t op_max(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t op_or(uint32_t a, uint32_t b) { return a | b; }
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  WAVE_SCAN(v, op_add);
  return v;
}
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
  WAVE_SCAN(v, op_max);
  return v;
}
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {  // uniform result
  WAVE_SCAN(v, op_or);
  return __builtin_amdgcn_readlane(v, 63);
}

// Exclusive scan across a workgroup of NT threads (NT/64 words of `sm`).
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *sm,
                                                    uint32_t *total) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  uint32_t inc = wave_incl_scan(v);
  if (lane == 63) sm[wid] = inc;
  __syncthreads();
  uint32_t wpre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    uint32_t s = sm[w];
    if (w < wid) wpre += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return wpre + inc - v;
}

// Exclusive scan of v and sum of w across the workgroup in one exchange.
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan_sum(uint32_t v, uint32_t w, uint32_t *sm,
                                                        uint32_t *total_v, uint32_t *total_w) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const uint32_t inc = wave_incl_scan(v);
  const uint32_t ws = __builtin_amdgcn_readlane(wave_incl_scan(w), 63);
  if (lane == 63) {
    sm[wid] = inc;
    sm[NT / 64 + wid] = ws;
  }
  __syncthreads();
  uint32_t wpre = 0, tv = 0, tw = 0;
#pragma unroll
  for (int k = 0; k < NT / 64; ++k) {
    const uint32_t x = sm[k];
    if (k < wid) wpre += x;
    tv += x;
    tw += sm[NT / 64 + k];
  }
  __syncthreads();
  *total_v = tv;
  *total_w = tw;
  return wpre + inc - v;
}

// Byte-stream writer for decode output: packs bytes into aligned 32-bit
// words; partial words at the two ends go out byte by byte, so neighbouring
// strings never overwrite each other's bytes.
struct ByteOut {
  uint8_t *p;
  uint32_t w, k;
  __device__ __forceinline__ void init(uint8_t *q) { p = q; w = 0; k = 0; }
  __device__ __forceinline__ void flush() {
    for (uint32_t i = 0; i < k; ++i) p[i] = (uint8_t)(w >> (8 * i));
    p += k; w = 0; k = 0;
  }
  __device__ __forceinline__ void put(uint32_t b) {
    w |= b << (8 * k);
    ++k;
    if ((((uintptr_t)p + k) & 3u) == 0) {
      if (k == 4) {
        *reinterpret_cast<uint32_t *>(p) = w;
        p += 4; w = 0; k = 0;
      } else {
        flush();
      }
    }
  }
};

// Address-space-explicit pointers, so LDS staging compiles to ds_* and
// global output to global_* (never flat_*).
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
// byte-aligned views for unaligned global stores (gfx950 takes them whole)
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef u32x4 __attribute__((aligned(1))) u32x4u;
typedef u32x2 __attribute__((aligned(1))) u32x2u;
typedef uint32_t __attribute__((aligned(1))) u32u;
typedef uint16_t __attribute__((aligned(1))) u16u;

// Word writer for encode output: the stream [o, o+E) receives big-endian
// 32-bit groups; with phase = o & 3 fixed, each group completes one aligned
// word (funnel shift with the pending bytes).  The head word that also holds
// the previous string's bytes, and the tail, are written byte by byte.

// 4 bytes at an arbitrary pool position, big-endian (first byte in bits
// 31..24); bytes at or past `end` read as zero.  Reads stay within
// align_up(end, 16) + 4 (pool padding contract).
__device__ __forceinline__ uint32_t load_be32(const uint8_t *base, uint32_t pos, uint32_t end) {
  const uint32_t a = pos & ~3u;
  const uint32_t w0 = *reinterpret_cast<const uint32_t *>(base + a);
  const uint32_t w1 = *reinterpret_cast<const uint32_t *>(base + a + 4);
  uint32_t x = __builtin_bswap32(__builtin_amdgcn_alignbyte(w1, w0, pos & 3u));
  const uint32_t v = end - pos;
  if (v < 4) x &= ~(0xFFFFFFFFu >> (8 * v));
  return x;
}


// The library's one source compiles as two translation units (Makefile):
// HD_PART_ENC (encode, string literals, scans, the C ABI for them) with the
// default instruction scheduler, and HD_PART_DEC (the decoders) with
// -amdgpu-sched-strategy=max-ilp, which shortens the decoders' dependent
// lookup chains (config 3 decode 300.4 vs 307.9 us) but slows the encode
// pack (146.3 vs 135.1).  With neither defined it is the whole library.
#ifndef HD_PART_DEC
// ---------------------------------------------------------------------------
// encode, pass 1: per-string encoded length  (lib/nghttp2_hd_huffman.c:34-43)
// ---------------------------------------------------------------------------

// decode slots: cap_i = floor(8 E_i / 5) + 1 (lib/nghttp2_hd_huffman.h:76-78)
__global__ __launch_bounds__(WG) void k_slot_len(const uint32_t *__restrict__ off, uint32_t n,
                                                 uint32_t *__restrict__ out_len,
                                                 uint32_t *__restrict__ tile_sums) {
  __shared__ uint32_t red[WG / 64];
  const uint32_t s = blockIdx.x * WG + threadIdx.x;
  uint32_t c = 0;
  if (s < n) {
    const uint32_t e = off[s + 1] - off[s];
    c = (uint32_t)(((uint64_t)e * 8u) / 5u) + 1u;
    out_len[s] = c;
  }
  uint32_t tot;
  block_excl_scan<WG>(c, red, &tot);
  if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
}

// Exclusive scan of the tile sums in place (4 per thread per round); writes
// the grand total to *grand (== offsets[n]).
__global__ __launch_bounds__(SCAN_WG) void k_scan_tiles(uint32_t *__restrict__ tile_sums,
                                                        uint32_t ntiles,
                                                        uint32_t *__restrict__ grand) {
  __shared__ uint32_t sm[SCAN_WG / 64];
  uint32_t carry = 0;
  for (uint32_t base = 0; base < ntiles; base += 4 * SCAN_WG) {
    const uint32_t i0 = base + 4 * threadIdx.x;
    uint32_t v[4], sum = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = (i0 + j < ntiles) ? tile_sums[i0 + j] : 0u;
      sum += v[j];
    }
    uint32_t tot;
    uint32_t run = carry + block_excl_scan<SCAN_WG>(sum, sm, &tot);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (i0 + j < ntiles) tile_sums[i0 + j] = run;
      run += v[j];
    }
    carry += tot;
  }
  if (threadIdx.x == 0) *grand = carry;
}

// in-place: offs[s] holds a length on entry, the exclusive prefix on exit
__global__ __launch_bounds__(WG) void k_scan_apply(uint32_t *__restrict__ offs, uint32_t n,
                                                   const uint32_t *__restrict__ tile_prefix) {
  __shared__ uint32_t red[WG / 64];
  const uint32_t s = blockIdx.x * WG + threadIdx.x;
  const uint32_t len = (s < n) ? offs[s] : 0u;
  uint32_t tot;
  const uint32_t o = tile_prefix[blockIdx.x] + block_excl_scan<WG>(len, red, &tot);
  if (s < n) offs[s] = o;
}

#define ENC_WAVES 4                  // waves per encode workgroup (tile = 256 strings)
#ifndef EC_STORE4
#define EC_STORE4 1  // k_encode: an interior round of <= 256 words as four unconditional stores
#endif
#ifndef EC_INTERIOR
#define EC_INTERIOR 1  // k_encode: interior rounds store their words without edge tests
#endif
#ifndef EC_CNT_SPLIT
#define EC_CNT_SPLIT 1  // the count's in-chunk prefixes in two halves (16-byte lane stride)
#endif
#ifndef EC_CNT_UNROLL
#define EC_CNT_UNROLL 1  // the count's wave loop: two chunk buffers, unrolled by two
#endif
#ifndef EC_CNT_PFD
#define EC_CNT_PFD 2  // k_enc_count: rounds of chunks in flight per wave (4: no faster)
#endif

// bytes of the 7-bit-prefix integer n (count_encoded_length(n, 7))
__device__ __forceinline__ uint32_t prefix7_len(uint32_t n) {
  if (n < 127u) return 1u;
  n -= 127u;
  uint32_t len = 2u;
  for (; n >= 128u; n >>= 7) ++len;
  return len;
}
// byte r of the literal's prefix (encode_length(buf, n, 7) with buf[0] = H)
__device__ __forceinline__ uint32_t prefix7_byte(uint32_t n, uint32_t h, uint32_t r) {
  if (r == 0) return (h << 7) | (n < 127u ? n : 127u);
  const uint32_t m = (n - 127u) >> (7u * (r - 1u));
  return (m & 0x7Fu) | (m >= 128u ? 0x80u : 0u);
}


// ---------------------------------------------------------------------------
// encode over aligned chunks (the product path): a wave owns 64 consecutive
// strings, i.e. the contiguous raw bytes [A, Z), and walks them as aligned
// 16-byte chunks, 64 per round (one per lane), whatever the string lengths.
// ---------------------------------------------------------------------------

// Pass 1 (lib/nghttp2_hd_huffman.c:34-43): code bits per string.  With P(x)
// = the code bits of the wave's bytes from its first chunk up to byte x, a
// string's bits are P(b) - P(a): each lane sums its chunk's code lengths
// (in-chunk exclusive prefixes to LDS, 16 bits a byte), a wave scan places
// the chunks, and every string lane reads P at its two ends.  Bytes before
// A or past Z in the edge chunks add the same amount to both ends.
// FR (emit_string, lib/nghttp2_hd.c:1001-1044): the tile sums are of the
// string LITERALS' bytes, prefix7_len(P) + P with P = min(E, R) (H = E < R).
// The code bits of a wave's 64 strings (string l in lane l: bytes [a_l,
// b_l)): each lane sums its aligned 16-byte chunk's code lengths (lenT in
// LDS, one byte per entry) and writes its in-chunk prefixes (16 bits a byte)
// to the wave's LDS scratch pr (512 words); one wave scan places the chunks,
// and every string lane reads P at its two ends.  Shared by k_enc_count and
// the single-tile k_encode.
__device__ __forceinline__ uint32_t wave_string_bits(const uint8_t *__restrict__ src, uint32_t a_l,
                                                     uint32_t b_l, bool sl, uint32_t nstr,
                                                     const lds_u8 *lenT, lds_u32 *pr, uint32_t lane) {
  const uint32_t A = __builtin_amdgcn_readfirstlane(a_l);
  const uint32_t Z = __builtin_amdgcn_readlane(b_l, nstr - 1u);
  const uint32_t c0 = A >> 4, c_end = (Z + 15u) >> 4;
  const lds_u16 *pr16 = (const lds_u16 *)pr;
  uint32_t Rc = 0, Pa = 0, Pb = 0;
  bool ga = false, gb = false;
  // one round: the 64 chunks from chunk cb, this lane's in qv
  auto round = [&](uint32_t cb, const uint4 &qv, bool ok) {
    const uint32_t base = cb << 4;
    const uint32_t wd[4] = {ok ? qv.x : 0u, ok ? qv.y : 0u, ok ? qv.z : 0u, ok ? qv.w : 0u};
    uint32_t run = 0, pk[8];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t L = lenT[(wd[j >> 2] >> (8 * (j & 3))) & 0xFFu];
      if (j & 1) pk[j >> 1] |= run << 16; else pk[j >> 1] = run;
      run += L;
    }
    u32x4 v0, v1;
    v0.x = pk[0]; v0.y = pk[1]; v0.z = pk[2]; v0.w = pk[3];
    v1.x = pk[4]; v1.y = pk[5]; v1.z = pk[6]; v1.w = pk[7];
#if EC_CNT_SPLIT
    // (the chunk's first and second 8 prefixes in two halves of pr: lane
    // strides of 16 bytes, 4-way per 32 lanes -- the least 16-byte stores
    // can take -- instead of 32 bytes, 8-way.  Round 6: count 34.9 vs 37.0
    // us on config 3, 14.4 vs 15.2 on config 2, outputs equal;
    // profiles/r06/ab/ab_count_split_prefixes.log)
    *(lds_u32x4 *)(pr + 4u * lane) = v0;
    *(lds_u32x4 *)(pr + 256u + 4u * lane) = v1;
#else
    *(lds_u32x4 *)(pr + 8u * lane) = v0;
    *(lds_u32x4 *)(pr + 8u * lane + 4u) = v1;
#endif
    const uint32_t Sinc = wave_incl_scan(run), Sx = Sinc - run;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the string ends in this round: P = chunk start + in-chunk prefix
    const uint32_t ra = a_l - base, rb = b_l - base;
    const uint32_t xa = __shfl(Sx, (ra >> 4) & 63u, 64), xb = __shfl(Sx, (rb >> 4) & 63u, 64);
    if (sl && ra < 1024u) {
      Pa = Rc + xa + pr16[EC_CNT_SPLIT ? ((ra >> 4) << 3) | (ra & 7u) | ((ra & 8u) << 6) : ra];
      ga = true;
    }
    if (sl && rb < 1024u) {
      Pb = Rc + xb + pr16[EC_CNT_SPLIT ? ((rb >> 4) << 3) | (rb & 7u) | ((rb & 8u) << 6) : rb];
      gb = true;
    }
    Rc += __builtin_amdgcn_readlane(Sinc, 63);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  // every lane loads (a chunk past the wave's bytes at a clamped index,
  // used as zeros): a load behind a branch that a whole wave may skip makes
  // the count of loads in flight path-dependent, and the compiler then waits
  // for all of them (vmcnt(0)) where it needs the oldest
  const uint32_t c_last = max(c_end, c0 + 1u) - 1u;
  auto load = [&](uint32_t c, bool &ok) -> uint4 {
    ok = c < c_end;
    return *reinterpret_cast<const uint4 *>(src + ((size_t)min(c, c_last) << 4));
  };
#if EC_CNT_UNROLL
  // chunks two rounds ahead, in two buffers the loop (unrolled by two)
  // alternates: a buffer is reloaded only after its round has used it, so
  // no register copy of a load in flight makes the round wait for it.
  // (Round 6: the rolled loop below rotated q[0] <- q[1] each round, and
  // that copy of the load just issued waited for it, vmcnt(0) -- every
  // round took a whole memory latency, whatever EC_CNT_PFD was.  Unrolled:
  // count 37.1 vs 40.9 us on config 3, encode pair 123.4 vs 127.8, config
  // 2 count 14.9 vs 15.4, outputs equal; profiles/r06/ab/ab_count_unroll.log)
  bool oka, okb;
  uint4 qa = load(c0 + lane, oka), qb = load(c0 + 64u + lane, okb);
  for (uint32_t cb = c0; cb < c_end; cb += 128u) {
    round(cb, qa, oka);
    qa = load(cb + 128u + lane, oka);
    if (cb + 64u >= c_end) break;
    round(cb + 64u, qb, okb);
    qb = load(cb + 192u + lane, okb);
  }
#else
  // chunks are loaded EC_CNT_PFD rounds ahead
  uint4 q[EC_CNT_PFD];
#pragma unroll
  for (uint32_t d = 0; d < EC_CNT_PFD; ++d) {
    q[d] = make_uint4(0, 0, 0, 0);
    if (c0 + 64u * d + lane < c_end) q[d] = *reinterpret_cast<const uint4 *>(src + ((c0 + 64u * d + lane) << 4));
  }
  for (uint32_t cb = c0; cb < c_end; cb += 64u) {
    const uint4 qv = q[0];
#pragma unroll
    for (uint32_t d = 0; d + 1 < EC_CNT_PFD; ++d) q[d] = q[d + 1];
    q[EC_CNT_PFD - 1] = make_uint4(0, 0, 0, 0);
    if (cb + 64u * EC_CNT_PFD + lane < c_end)
      q[EC_CNT_PFD - 1] = *reinterpret_cast<const uint4 *>(src + ((cb + 64u * EC_CNT_PFD + lane) << 4));
    round(cb, qv, true);
  }
#endif
  // an end at the last chunk's end (Z on a chunk boundary)
  if (!ga) Pa = Rc;
  if (!gb) Pb = Rc;
  return sl ? Pb - Pa : 0u;
}

// k_enc_count: strings per wave (a tile of 256 is 256 / SPW waves); 32 / 16
// measured slower (config 3 encode pair 137.5 / 146.3 vs 135.8 us)
#define EC_CNT_SPW 64u
#define EC_CNT_NT (WG * 64u / EC_CNT_SPW)
template <bool FR>
__global__ __launch_bounds__(EC_CNT_NT) void k_enc_count(const uint8_t *__restrict__ src,
                                                  const uint32_t *__restrict__ off,
                                                  uint32_t n,
                                                  uint32_t *__restrict__ out_len,
                                                  uint32_t *__restrict__ tile_sums,
                                                  int bits_out) {
  __shared__ uint8_t lenT[256];
  __shared__ alignas(16) uint32_t pre[EC_CNT_NT / 64][512];  // a round's prefixes (u16 per byte)
  __shared__ uint32_t red[2 * EC_CNT_NT / 64];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  if (threadIdx.x < 256) lenT[threadIdx.x] = dev::hd_huff_enc_len[threadIdx.x];
  __syncthreads();
  const uint32_t t0 = blockIdx.x * WG + EC_CNT_SPW * wv;  // the wave's strings
  uint32_t e = 0;
  bool huge = false;
  if (t0 < n) {
    const uint32_t nstr = min(n - t0, EC_CNT_SPW);
    const bool sl = lane < nstr;
    const uint32_t a_l = sl ? off[t0 + lane] : 0u, b_l = sl ? off[t0 + lane + 1] : 0u;
    huge = b_l - a_l > NGHTTP2_AMD_ENCODE_MAX_STRING;
    const uint32_t bits = wave_string_bits(src, a_l, b_l, sl, nstr, (const lds_u8 *)lenT,
                                           (lds_u32 *)pre[wv], lane);
    e = (bits + 7u) >> 3;
    if (sl && out_len) out_len[t0 + lane] = bits_out ? bits : e;
    if (FR && sl) {
      const uint32_t R = b_l - a_l, P = e < R ? e : R;
      e = prefix7_len(P) + P;
    }
  }
  if (tile_sums) {
    uint32_t tot, hi;
    // a string whose code bits would not fit the 32-bit counts, or a tile
    // whose output may reach 2^29 bytes (its sum in 64 KiB units, which
    // cannot wrap, within 256 units of 2^13: k_encode places a wave's bits
    // in 32-bit positions), poisons its tile's sum (0xFFFFFFFF), so this tile
    // and every one after it overflow in k_encode.  (Round 4: 64-bit bit
    // positions in k_encode instead cost 8.7 us of 140 on config 3.)
    block_excl_scan_sum<EC_CNT_NT>(e, huge ? 0x2000u : e >> 16, red, &tot, &hi);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = hi >= 0x2000u - WG ? 0xFFFFFFFFu : tot;
  }
}

// Pass 2 (lib/nghttp2_hd_huffman.c:45-104): bit packing.  The EOS-prefix
// padding of a string (:95-101, pad = 8 E - bits, known from pass 1) is
// counted as extra length of its last byte's code (codes are MSB-aligned, so
// the pad is just zero bits after the code), so the bit stream of the wave
// is the plain concatenation of every byte's code and every string's pad,
// and a chunk starts at the wave scan of the chunk lengths -- no per-byte
// alignment.  A lane combines its 16 codes in registers (pairs of < 32
// bits, then quads of < 64) and ORs each quad into the round's LDS image
// (three words); a round with a longer pair goes byte by byte.  The pad
// bits themselves are all ones, OR'ed in by the string's own lane.  The
// image goes out as whole big-endian dwords (the dwords at the wave's two
// ends bytewise), the partial last word carried into the next round.  The
// first chunk's bytes before A are placed before the wave's first bit, in
// a margin of the image that is never stored.
// The tile sums' exclusive 64-bit prefix for a large batch (one workgroup):
// past EC_SCAN_TILES tiles, k_encode's own sum of the tiles before it (each
// workgroup reads all of them, O(tiles^2) L2 reads: 8.6 GB for 16M strings)
// costs more than this launch.  A poisoned tile (0xFFFFFFFF) pushes every
// later prefix past the uint32 offsets, as the in-kernel sum does.
#ifndef EC_SCAN_TILES
#define EC_SCAN_TILES 16384u
#endif
__global__ __launch_bounds__(1024) void k_tile_prefix64(const uint32_t *__restrict__ tiles, uint32_t nt,
                                                        uint64_t *__restrict__ pre) {
  __shared__ uint64_t wsum[16];
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t per = (nt + 1023u) / 1024u, b = min(t * per, nt), e = min(b + per, nt);
  uint64_t s = 0;
  for (uint32_t i = b; i < e; ++i) s += tiles[i];
  uint64_t inc = s;
#pragma unroll
  for (uint32_t d = 1; d < 64u; d <<= 1) {
    const uint64_t v = __shfl_up(inc, d, 64);
    if (lane >= d) inc += v;
  }
  if (lane == 63u) wsum[wv] = inc;
  __syncthreads();
  uint64_t run = inc - s;
  for (uint32_t w = 0; w < wv; ++w) run += wsum[w];
  for (uint32_t i = b; i < e; ++i) {
    pre[i] = run;
    run += tiles[i];
  }
}

#ifndef EC_WPE
#define EC_WPE 4  // k_encode: waves per SIMD the register budget is sized for
#endif
#define EC_M 16u                    // image margin (words): >= 15 bytes x 30 bits
#define EC_RW (EC_M + 1024u + 32u)  // + 1 KB at <= 32 bits a byte + carry + bytes past Z
// FR: + the wave's literal prefixes and pads (64 x (6 x 8 + 7) bits)
#define EC_RW_F (EC_RW + 112u)

// OR the MSB-aligned bits {hi, lo} into the image at bit b
__device__ __forceinline__ void ec_or3(lds_u32 *img, uint32_t b, uint32_t hi, uint32_t lo,
                                       uint32_t rw = 0xFFFFFFFFu) {
  HD_CHECK((b >> 5) + 2u < rw, 0x101u);
  (void)rw;
  const uint32_t o = b & 31u;
  lds_u32 *q = img + (b >> 5);
  atomicOr((uint32_t *)&q[0], hi >> o);
  atomicOr((uint32_t *)&q[1], __builtin_amdgcn_alignbit(hi, lo, o));
  atomicOr((uint32_t *)&q[2], __builtin_amdgcn_alignbit(lo, 0u, o));  // (0 when o = 0)
}

// FR: emit_string (lib/nghttp2_hd.c:1001-1044) fused into the pack -- every
// string leaves as its HPACK string literal, back to back in wire order:
// the prefix (H bit, 7-bit-prefix length of P = min(E, R), :823-863) and the
// Huffman payload (H = E < R) or the raw bytes.  In the wave's bit stream a
// literal's prefix bits are extra length attached to the input byte before
// the string (the previous string's last byte; at the wave start, an initial
// offset), so the stream stays the concatenation of the bytes' codes (raw
// strings: the byte itself, 8 bits) and the extra bits; the prefix values
// and the pads' ones are OR'ed in by the string's own lane.  Extras reach
// tens of bits, so FR combines codes in 64-bit pairs (not 32-bit pairs and
// quads) and keeps the per-byte extras as u16.
// ONE: a batch of one tile (n <= 256) in a single launch -- the code bits
// and the tile's total are counted in this workgroup first (the count
// kernel's wave loop, its LDS scratch in the image), so a small batch (the
// drop-in's single string, a deflater's header list) pays one launch, not two
template <bool FR, bool ONE = false>
__global__ __launch_bounds__(WG, EC_WPE) void k_encode(const uint8_t *__restrict__ src,
                                               const uint32_t *__restrict__ off, uint32_t n,
                                               uint8_t *__restrict__ dst, uint64_t dst_cap,
                                               uint32_t *__restrict__ dst_off,
                                               const uint32_t *__restrict__ tile_sums,
                                               const uint64_t *__restrict__ tile_pre) {
  constexpr uint32_t RW = FR ? EC_RW_F : EC_RW;
  constexpr uint32_t PDW = FR ? 512u : 256u;  // u16 extras / u8 pads per round byte
  __shared__ uint2 codeT[256];  // {code MSB-aligned, length}
  __shared__ uint32_t image[ENC_WAVES][RW];
  __shared__ alignas(16) uint32_t padb[ENC_WAVES][PDW];  // a round's pad bits (u8 per byte)
  __shared__ uint32_t rawm[ENC_WAVES][FR ? 32 : 1];       // FR: a round's raw-string bytes
  __shared__ uint32_t o_sh[WG + 1];
  __shared__ uint32_t red[2 * (WG / 64)];
  __shared__ uint8_t lenT1[ONE ? 256 : 1];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  // every load of the prologue is issued before any is used, so a tile's
  // start costs one memory latency (round 5: the staging, the offsets, the
  // tile sums and the tile's own sum waited in turn)
  const uint32_t s_me = blockIdx.x * WG + threadIdx.x;
  const uint32_t t0 = blockIdx.x * WG + 64u * wv;
  const uint32_t nstr = t0 < n ? min(n - t0, 64u) : 0u;
  const bool sl = lane < nstr;
  const uint32_t a_l = sl ? off[t0 + lane] : 0u, b_l = sl ? off[t0 + lane + 1] : 0u;
  uint32_t bits_me, tsum;
  if constexpr (ONE) {
    lenT1[threadIdx.x] = dev::hd_huff_enc_len[threadIdx.x];
    __syncthreads();
    bits_me = nstr ? wave_string_bits(src, a_l, b_l, sl, nstr, (const lds_u8 *)lenT1,
                                      (lds_u32 *)image[wv], lane)
                   : 0u;
    // the tile's total and its poison, as k_enc_count computes them
    uint32_t e1 = (bits_me + 7u) >> 3;
    if (FR && sl) {
      const uint32_t R = b_l - a_l, P = e1 < R ? e1 : R;
      e1 = prefix7_len(P) + P;
    }
    const bool huge = b_l - a_l > NGHTTP2_AMD_ENCODE_MAX_STRING;
    uint32_t tot1, hi1;
    block_excl_scan_sum<WG>(sl ? e1 : 0u, huge ? 0x2000u : (sl ? e1 : 0u) >> 16, red, &tot1, &hi1);
    tsum = hi1 >= 0x2000u - WG ? 0xFFFFFFFFu : tot1;
  } else {
    bits_me = s_me < n ? dst_off[s_me] : 0u;
    tsum = tile_sums[blockIdx.x];
  }
  const uint32_t cc = dev::hd_huff_enc_code[threadIdx.x], cl = dev::hd_huff_enc_len[threadIdx.x];
  // the tile's offset: the tile totals before it (k_enc_count; 16 KB for 1M
  // strings, L2-resident), in 64 bits (a batch's encoded total may pass the
  // uint32 offset range); pre is each thread's part of the sum the block
  // scans add up.  Thread t sums tiles [16 t, 16 t + 16) of each 4096 before
  // this one with four 16-byte loads issued together (round 5: a strided
  // loop that waited for each load in turn, 29 % of a wave's time on config
  // 3 by the stamps)
  uint64_t pre = 0;
  const uint32_t bt = blockIdx.x;
  const bool vec = tile_pre == nullptr && ((uintptr_t)tile_sums & 15u) == 0;
  uint4 v[4];
  auto batch_load = [&](uint32_t base) {
    const uint32_t q0 = base + 16u * threadIdx.x;
#pragma unroll
    for (uint32_t k = 0; k < 4u; ++k)
      v[k] = q0 + 4u * k < bt ? reinterpret_cast<const uint4 *>(tile_sums)[(q0 >> 2) + k] : make_uint4(0, 0, 0, 0);
  };
  auto batch_sum = [&](uint32_t base) {
    const uint32_t q0 = base + 16u * threadIdx.x;
#pragma unroll
    for (uint32_t k = 0; k < 4u; ++k) {
      const uint32_t i = q0 + 4u * k;  // (the 16 bytes may reach 3 tiles past bt: masked)
      pre += (uint64_t)(i < bt ? v[k].x : 0u) + (i + 1u < bt ? v[k].y : 0u) +
             (uint64_t)(i + 2u < bt ? v[k].z : 0u) + (i + 3u < bt ? v[k].w : 0u);
    }
  };
  if (tile_pre) {  // the prefixes were scanned by k_tile_prefix64 (every thread reads its tile's)
    pre = tile_pre[bt];
  } else if (vec) {
    batch_load(0u);
  }
  codeT[threadIdx.x] = make_uint2(cc, cl);
  lds_u32 *img = (lds_u32 *)image[wv];
  for (uint32_t i = lane; i < RW; i += 64u) img[i] = 0u;
  lds_u32 *pdw = (lds_u32 *)padb[wv];
  lds_u8 *pdb = (lds_u8 *)padb[wv];
  lds_u16 *pdh = (lds_u16 *)padb[wv];
  lds_u32 *rwm = (lds_u32 *)rawm[wv];
#pragma unroll
  for (uint32_t i = 0; i < PDW / 64u; ++i) pdw[lane + 64u * i] = 0u;
  // (thread s_me is lane `lane` of string t0 + lane)
  const uint32_t Eh_me = (bits_me + 7u) >> 3;  // Huffman bytes
  const uint32_t R_me = b_l - a_l;
  const bool H_me = FR && Eh_me < R_me;        // FR: the literal is Huffman-coded
  const uint32_t P_me = FR ? (H_me ? Eh_me : R_me) : 0u;
  const uint32_t PL_me = FR && sl ? prefix7_len(P_me) : 0u;
  const uint32_t E_me = FR ? (sl ? PL_me + P_me : 0u) : Eh_me;  // output bytes of string s_me
  const uint32_t A = __builtin_amdgcn_readfirstlane(a_l);
  const uint32_t Z = nstr ? __builtin_amdgcn_readlane(b_l, nstr - 1u) : 0u;
  const uint32_t c0 = A >> 4, c_end = (Z + 15u) >> 4;
  uint4 wn = make_uint4(0, 0, 0, 0);  // the next round's chunk (prefetched)
  if (c0 + lane < c_end) wn = *reinterpret_cast<const uint4 *>(src + ((c0 + lane) << 4));
  if (vec) {
    batch_sum(0u);
    for (uint32_t base = 16u * WG; base < bt; base += 16u * WG) {  // (past 4096 tiles)
      batch_load(base);
      batch_sum(base);
    }
  } else if (!tile_pre) {
    for (uint32_t t = threadIdx.x; t < bt; t += WG) pre += tile_sums[t];
  }
  uint32_t tot32, ptot_lo, ptot_hi = 0;
  // the 64-bit prefix as two 32-bit sums: 256 parts of 23 bits fit 31 bits
  // (tile_pre: every thread holds the whole prefix, no sum)
  const uint32_t loc = block_excl_scan_sum<WG>(E_me, tile_pre ? 0u : (uint32_t)(pre & 0x7FFFFFu), red, &tot32,
                                               &ptot_lo);  // (barriers)
  // (a string too long for the 32-bit code-bit counts poisoned the tile's
  // sum: the tile overflows)
  const uint64_t tot = tsum == 0xFFFFFFFFu ? 0x100000000ull : (uint64_t)tot32;
  if (!tile_pre) {
    uint32_t dummy;
    block_excl_scan_sum<WG>(0u, (uint32_t)(pre >> 23), red, &dummy, &ptot_hi);
  }
  const uint64_t ptot = tile_pre ? pre : ((uint64_t)ptot_hi << 23) + ptot_lo;
  // uint32 offsets: a tile whose strings would end past the limit writes no
  // bytes, saturated offsets and the overflow mark in dst_off[n]
  const uint64_t limit = dst_cap < 0xFFFFFFFEull ? dst_cap : 0xFFFFFFFEull;
  if (ptot + tot > limit) {
    if (s_me < n) dst_off[s_me] = (uint32_t)min(ptot + loc, limit);
    if (s_me == n - 1u) dst_off[n] = NGHTTP2_AMD_OFF_OVERFLOW;
    return;
  }
  const uint32_t o_me = (uint32_t)ptot + loc;
  if (s_me < n) dst_off[s_me] = o_me;
  if (s_me == n - 1u) dst_off[n] = o_me + E_me;
  o_sh[threadIdx.x] = o_me;
  if (threadIdx.x == WG - 1) o_sh[WG] = o_me + E_me;
  __syncthreads();
  if (nstr == 0) return;
  // the wave's output bytes (EC_STORE4, the pack: as scalars, so the
  // round's word bounds and path choices stay scalar)
  const uint32_t OA = EC_STORE4 && !FR ? __builtin_amdgcn_readfirstlane(o_sh[64u * wv]) : o_sh[64u * wv];
  const uint32_t OZ = EC_STORE4 && !FR ? __builtin_amdgcn_readfirstlane(o_sh[64u * wv + nstr])
                                       : o_sh[64u * wv + nstr];
  const uint64_t G0 = 8ull * OA;
  const uint32_t pad_l = sl && (!FR || H_me) ? 8u * Eh_me - bits_me : 0u;  // EOS-prefix bits after string l
  const uint32_t olast_l = o_me + E_me - 1u;             // its last output byte (if E > 0)
  const uint32_t tail_l = b_l - 1u;                      // its last raw byte
  // FR: the prefixes of the strings that start at the wave's first byte go
  // before it (an initial offset XS); every other string's prefix is extra
  // length of the byte before it; raw strings (any in the wave: anyraw) take
  // their bytes as 8-bit codes
  const bool at_a = FR && sl && a_l == A;
  const uint32_t XS = FR ? __builtin_amdgcn_readlane(wave_incl_scan(at_a ? 8u * PL_me : 0u), 63) : 0u;
  const bool rawl = FR && sl && !H_me && R_me > 0u;
  const bool anyraw = FR && __ballot(rawl) != 0;
  // (FR: a wave of empty strings only still has its literals: one round)
  const uint32_t c_stop = FR && c_end == c0 ? c0 + 1u : c_end;
  uint32_t x = 0;  // output bit of the round's first wave byte (relative to G0; a wave's
                   // output is below 2^32 bits: k_enc_count poisons a tile of 2^29 bytes)
  for (uint32_t cb = c0; cb < c_stop; cb += 64u) {
    const bool first = cb == c0, last_round = cb + 64u >= c_stop;
    const uint32_t base = cb << 4;
    const uint64_t WB = (G0 + x) >> 5;  // global word of img[EC_M]
    // ---- pads of the strings ending in this round, at their last raw byte
    const bool tl = sl && pad_l && b_l > a_l && tail_l - base < 1024u;
    // FR: my prefix as extra length of the byte before my string
    const bool pfx = FR && sl && a_l > A && a_l - 1u - base < 1024u;
    if (!FR) {
      if (tl) pdb[tail_l - base] = (uint8_t)pad_l;
    } else {
      if (tl) atomicAdd((uint32_t *)&pdw[(tail_l - base) >> 1], pad_l << (16u * ((tail_l - base) & 1u)));
      if (pfx) atomicAdd((uint32_t *)&pdw[(a_l - 1u - base) >> 1], (8u * PL_me) << (16u * ((a_l - 1u - base) & 1u)));
      if (anyraw) {
        if (lane < 32u) rwm[lane] = 0u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t lo = max(a_l, base), hi = min(b_l, base + 1024u);
        if (rawl && lo < hi) {
          for (uint32_t w = (lo - base) >> 5; w <= (hi - 1u - base) >> 5; ++w) {
            const uint32_t w0 = base + 32u * w;
            const uint32_t f = max(lo, w0) - w0, t = min(hi, w0 + 32u) - w0;  // bits [f, t)
            atomicOr((uint32_t *)&rwm[w], (t - f == 32u ? 0xFFFFFFFFu : ((1u << (t - f)) - 1u)) << f);
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t p0 = base + 16u * lane;
    const bool act = p0 < Z;  // (lanes past the wave's last chunk: nothing)
    const uint32_t wd[4] = {wn.x, wn.y, wn.z, wn.w};
    wn = make_uint4(0, 0, 0, 0);
    if (cb + 64u + lane < c_end) wn = *reinterpret_cast<const uint4 *>(src + p0 + 1024u);
#define EC_B8(j) (((j) & 3) ? (wd[(j) >> 2] >> (8 * ((j) & 3) - 3)) & 0x7F8u : (wd[(j) >> 2] << 3) & 0x7F8u)
    // (!FR) per input dword: four codes (+ the pad at a string's last byte)
    // -> two pairs {pc, pl} (MSB-aligned, < 32 bits) -> one quad {qh:qo, ql};
    // (FR) per byte pair: {ph:po} (MSB-aligned, <= 64 bits), length pq
    uint32_t pd[FR ? 8 : 4];
    {
      const u32x4 pdv = *(const lds_u32x4 *)(pdw + (FR ? 8u : 4u) * lane);
      pd[0] = pdv.x; pd[1] = pdv.y; pd[2] = pdv.z; pd[3] = pdv.w;
      if (FR) {
        const u32x4 pdv2 = *(const lds_u32x4 *)(pdw + 8u * lane + 4u);
        pd[4 % (FR ? 8 : 4)] = pdv2.x; pd[5 % (FR ? 8 : 4)] = pdv2.y;
        pd[6 % (FR ? 8 : 4)] = pdv2.z; pd[7 % (FR ? 8 : 4)] = pdv2.w;
      }
    }
    const uint32_t rm = FR && anyraw ? (rwm[lane >> 1] >> (16u * (lane & 1u))) & 0xFFFFu : 0u;
    // (FR) the first chunk's bytes before A take no bits: the wave-start
    // prefixes (XS) are the first bits of the image, stored
    const uint32_t km = FR && first && lane == 0u ? (1u << (A & 15u)) - 1u : 0u;
    uint32_t qh[FR ? 8 : 4], qo[FR ? 8 : 4], ql[FR ? 8 : 4], plx = 0;
    if (!FR) {
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        uint32_t c[4], l[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint2 cj = *(const uint2 *)((const char *)codeT + EC_B8(4 * m + u));
          c[u] = cj.x;
          l[u] = cj.y + ((pd[m] >> (8 * u)) & 0xFFu);
        }
        const uint32_t pl0 = l[0] + l[1], pl1 = l[2] + l[3];
        const uint32_t pc0 = c[0] | (c[1] >> l[0]), pc1 = c[2] | (c[3] >> l[2]);
        plx = max(plx, max(pl0, pl1));
        ql[m] = pl0 + pl1;
        qh[m] = pc0 | (pc1 >> pl0);
        qo[m] = __builtin_amdgcn_alignbit(pc1, 0u, pl0);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        uint32_t c[2], l[2], xt[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int j = 2 * k + u;
          const uint32_t b8 = EC_B8(j);
          const uint2 cj = *(const uint2 *)((const char *)codeT + b8);
          const bool raw = (rm >> j) & 1u, skip = (km >> j) & 1u;
          c[u] = skip ? 0u : raw ? b8 << 21 : cj.x;  // a raw byte: itself, MSB-aligned
          l[u] = skip ? 0u : raw ? 8u : cj.y;
          xt[u] = (pd[k % (FR ? 8 : 4)] >> (16 * u)) & 0xFFFFu;
        }
        const uint32_t L0 = l[0] + xt[0];  // c1 starts L0 bits after c0
        const uint64_t v = ((uint64_t)c[1] << 32) >> (L0 & 63u);
        plx = max(plx, L0 + l[1]);
        qh[k % (FR ? 8 : 4)] = c[0] | (uint32_t)(v >> 32);
        qo[k % (FR ? 8 : 4)] = (uint32_t)v;
        ql[k % (FR ? 8 : 4)] = L0 + l[1] + xt[1];
      }
    }
    uint32_t S = 0;
#pragma unroll
    for (int m = 0; m < (FR ? 8 : 4); ++m) S += ql[m];
    S = act ? S : 0u;
    // a pair of 32 (FR: 64) bits or more: bytewise
    const bool longp = __ballot(act && plx > (FR ? 64u : 31u)) != 0;
    // ---- the first chunk's bytes before A go before the wave's first bit
    // (no pads there)
    uint32_t RA = 0;
    if (!FR && first) {
      const uint32_t k = A & 15u;
      uint32_t ra = 0;
#pragma unroll
      for (int j = 0; j < 15; ++j)
        if ((uint32_t)j < k) ra += ((const uint2 *)((const char *)codeT + EC_B8(j)))->y;
      RA = __builtin_amdgcn_readfirstlane(ra);
    }
    const uint32_t Sinc = wave_incl_scan(S);
    const uint32_t X0 = first ? XS : 0u;  // (FR) the wave-start prefixes
    // my chunk's first bit in the image (img[0] = global word WB - EC_M)
    const uint32_t ib0 = (uint32_t)(G0 + x - 32ull * WB) + 32u * EC_M + (Sinc - S) + X0 - RA;
    if (act) {
      if (!longp) {
        uint32_t b = ib0;
#pragma unroll
        for (int m = 0; m < (FR ? 8 : 4); ++m) {
          ec_or3(img, b, qh[m], qo[m], RW);
          b += ql[m];
        }
      } else {  // a code of <= 37 bits, MSB-aligned in 64; one dword at a time
        uint32_t b = ib0;
#pragma unroll 1
        for (uint32_t m = 0; m < 4u; ++m) {
          const uint32_t w = m == 0 ? wd[0] : m == 1 ? wd[1] : m == 2 ? wd[2] : wd[3];
          const uint32_t pw = m == 0 ? pd[0] : m == 1 ? pd[1] : m == 2 ? pd[2] : pd[3 % (FR ? 8 : 4)];
          const uint32_t pw2 = FR ? (m == 0 ? pd[1] : m == 1 ? pd[3] : m == 2 ? pd[5 % (FR ? 8 : 4)]
                                                                          : pd[7 % (FR ? 8 : 4)]) : 0u;
          const uint32_t pwf = FR ? (m == 0 ? pd[0] : m == 1 ? pd[2] : m == 2 ? pd[4 % (FR ? 8 : 4)]
                                                                          : pd[6 % (FR ? 8 : 4)]) : pw;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const uint32_t b8 = u ? (w >> (8 * u - 3)) & 0x7F8u : (w << 3) & 0x7F8u;
            const uint2 cj = *(const uint2 *)((const char *)codeT + b8);
            if (FR) {
              const bool raw = (rm >> (4u * m + u)) & 1u, skip = (km >> (4u * m + u)) & 1u;
              const uint32_t xw = u < 2 ? pwf : pw2;
              ec_or3(img, b, skip ? 0u : raw ? b8 << 21 : cj.x, 0u, RW);
              b += (skip ? 0u : raw ? 8u : cj.y) + ((xw >> (16 * (u & 1))) & 0xFFFFu);
            } else {
              ec_or3(img, b, cj.x, 0u, RW);
              b += cj.y + ((pw >> (8 * u)) & 0xFFu);
            }
          }
        }
      }
    }
#undef EC_B8
    // ---- EOS-prefix padding (all ones) of the strings that end in this round
    if (tl) {
      const uint32_t r = (uint32_t)((olast_l >> 2) - WB) + EC_M;
      HD_CHECK(r < RW, 0x102u);
      atomicOr((uint32_t *)&img[r], ((1u << pad_l) - 1u) << (24u - 8u * (olast_l & 3u)));
    }
    // ---- (FR) the literal prefixes attached in this round: H bit and the
    // 7-bit-prefix length (encode_length, lib/nghttp2_hd.c:823-863) at the
    // literal's first output bytes
    if (FR && (pfx || (first && at_a))) {
      for (uint32_t r = 0; r < PL_me; ++r) {
        const uint32_t q = o_me + r;
        const uint32_t v = prefix7_byte(P_me, H_me ? 1u : 0u, r);
        HD_CHECK((uint32_t)((q >> 2) - WB) + EC_M < RW, 0x103u);
        atomicOr((uint32_t *)&img[(uint32_t)((q >> 2) - WB) + EC_M], v << (24u - 8u * (q & 3u)));
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // ---- store whole words and zero them; carry a partial last word
    const uint32_t xe = last_round ? 8u * (OZ - OA) : x + __builtin_amdgcn_readlane(Sinc, 63) + X0 - RA;
    const uint32_t nw = (uint32_t)(((G0 + xe + 31u) >> 5) - WB);
    const uint32_t nst = last_round ? nw : (uint32_t)(((G0 + xe) >> 5) - WB);
    // words [ilo, ihi) lie inside the wave's output [OA, OZ) (<= dst_cap by
    // the tile check); the others hold bytes of the neighbouring waves
    const uint32_t ilo = (uint32_t)(((uint64_t)OA + 3u) / 4u - min(WB, ((uint64_t)OA + 3u) / 4u));
    const uint32_t ihi = (uint32_t)((uint64_t)OZ / 4u > WB ? (uint64_t)OZ / 4u - WB : 0u);
    uint8_t *const dw = dst + 4ull * WB;  // (uniform)
    HD_CHECK(EC_M + nw <= RW, 0x104u);
    HD_CHECK(ihi <= ilo || 4ull * (WB + ihi) <= dst_cap, 0x105u);
#if EC_INTERIOR
    // a round whose words all lie inside the wave's output (every round but
    // the first and the last, in practice): whole-word stores with no
    // per-word edge test (its exec-mask branches cost ~6 scalar
    // instructions per word and lane; round 6: config 3 encode pair 130.3
    // vs 135.0 us, emit 217.0 vs 223.6, config 2 flat, outputs equal;
    // profiles/r06/ab/ab_pack_interior_rounds.log)
    if (ilo == 0u && ihi >= nst) {
#if EC_STORE4
      // (EC_STORE4, the pack: a round of 1..256 words as exactly four store
      // instructions with no branch -- a lane past the round's words stores
      // the last word again, read before any word is cleared; the other
      // store paths end waiting for their stores.  Config 3 encode pair
      // 120.9 vs 122.9 us, config 2 flat; the string literals' config 2
      // 69.8 vs 68.0, so not for them; profiles/r06/ab/ab_pack_store4.log)
      if (EC_STORE4 && !FR && nst - 1u < 256u) {
        uint32_t v[4], ix[4];
#pragma unroll
        for (uint32_t k = 0; k < 4u; ++k) {
          ix[k] = min(lane + 64u * k, nst - 1u);
          v[k] = __builtin_bswap32(img[EC_M + ix[k]]);
        }
#pragma unroll
        for (uint32_t k = 0; k < 4u; ++k) img[EC_M + ix[k]] = 0u;
#pragma unroll
        for (uint32_t k = 0; k < 4u; ++k) *reinterpret_cast<uint32_t *>(dw + 4u * ix[k]) = v[k];
      } else
#endif
      {
        for (uint32_t i = lane; i < nst; i += 64u) {
          const uint32_t v = __builtin_bswap32(img[EC_M + i]);
          img[EC_M + i] = 0u;
          *reinterpret_cast<uint32_t *>(dw + 4u * i) = v;
        }
#if EC_STORE4
        if (!FR) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this path's stores, counted out
#endif
      }
    } else
#endif
    {
      for (uint32_t i = lane; i < nst; i += 64u) {
        const uint32_t v = __builtin_bswap32(img[EC_M + i]);
        img[EC_M + i] = 0u;
        if (i >= ilo && i < ihi) {
          *reinterpret_cast<uint32_t *>(dw + 4u * i) = v;
        } else {
          const uint64_t ga = 4ull * (WB + i);
          for (uint32_t y = 0; y < 4u; ++y) {
            const uint64_t gq = ga + y;
            if (gq >= OA && gq < OZ) dst[gq] = (uint8_t)(v >> (8u * y));
          }
        }
      }
#if EC_STORE4
      if (!FR) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
#endif
    }
    if (first && lane < EC_M) img[lane] = 0u;  // the bytes before A
    if (!FR) {
      if (tl) pdb[tail_l - base] = 0u;
    } else {
      if (tl) pdh[tail_l - base] = 0u;
      if (pfx) pdh[a_l - 1u - base] = 0u;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (!last_round && nst < nw) {  // the partial word moves to img[EC_M]
      const uint32_t cw = img[EC_M + nst];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (lane == 0) {
        img[EC_M + nst] = 0u;
        img[EC_M] = cw;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    x = xe;
  }
}

#endif  // !HD_PART_DEC
#ifndef HD_PART_ENC
// ---------------------------------------------------------------------------
// decode: canonical multi-symbol decoder
// ---------------------------------------------------------------------------
// Lookup entry (tools/gen_tables.py): sym1 | L1 << 8 | cnt << 13 | sym2 << 16 | used << 27
// (sym2 = 0 when cnt = 1).  The output bytes are bits 0..7 and 16..23 (E_OUT2):
// the item decoder stores the second with ds_write_b8_d16_hi, no shift (round
// 3; sym2 in bits 8..15 took a shift per entry).  A sink's put/put_nf take
// their bytes in that form.
#define E_CNT8(e) (((e) >> 10) & 0x18u)
#define E_CNT(e) (((e) >> 13) & 3u)
#define E_L1(e) (((e) >> 8) & 31u)
#define E_USED(e) ((e) >> 27)
#define E_OUT2 0x00FF00FFu
#define E_OUT1 0x000000FFu
#define E_EOS 0x00008000u  // (long-code entries only) the code is EOS
static_assert(HD_HUFF_LONG1_N0 == 12 && HD_HUFF_LONG1_ROWS == 20, "long-code table shape");
// The decoder's LDS tables for an LB-bit first-level lookup (14: 64 KB, the
// most two-symbol entries; 13: 32 KB, which leaves room for more waves).
template <int LB>
struct DecT {
  static constexpr int BITS = LB;
  uint32_t lut[1 << LB];
  // codes past the lookup by their leading ones (hd_huff_long1: n1 = 12..31,
  // then the 5 bits after the first zero), staged as lookup entries (one
  // symbol, used = its length) with E_EOS for the 30-bit EOS code
  uint32_t long1[HD_HUFF_LONG1_ROWS * 32];
  uint32_t depth_lo[30];
  uint16_t depth_base[30];
  uint8_t depth_ids[256];
};
static_assert(HD_HUFF_LUT_BITS == 14, "primary lookup");
typedef DecT<HD_HUFF_LUT_BITS> DecTables;

// (threads below `first` only meet the barrier: they may do other work,
// e.g. the item decoder's range search, while the rest stage)
template <int LB>
__device__ __forceinline__ void stage_dec_tables(DecT<LB> &T, uint32_t nthreads, uint32_t first = 0) {
  static_assert(LB == 13 || LB == 14, "lookup widths generated");
  const uint32_t t = threadIdx.x - first;  // (wraps above nthreads for threads below first)
  nthreads -= first;
  const uint32_t *lut = LB == 13 ? dev::hd_huff_lut13 : dev::hd_huff_lut;
  for (uint32_t i = t; i < (1u << LB); i += nthreads) T.lut[i] = lut[i];
  for (uint32_t i = t; i < HD_HUFF_LONG1_ROWS * 32u; i += nthreads) {
    const uint32_t v = dev::hd_huff_long1[i], sym = v & 511u, L = v >> 9;
    T.long1[i] = (sym & 255u) | (L << 8) | (1u << 13) | (L << 27) | (sym == 256u ? E_EOS : 0u);
  }
  if (t < 30) {
    T.depth_lo[t] = dev::hd_huff_depth_lo[t];
    T.depth_base[t] = dev::hd_huff_depth_base[t];
  }
  if (t < 256) T.depth_ids[t] = dev::hd_huff_depth_ids[t];
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Item decoding (DESIGN.md "decode").  A string of E encoded bytes is cut
// into m = max(1, ceil(E / P)) ITEMS, P = PIECE_BYTES = 64:
//   item (i, 0)   the string from its first bit (exact), up to the first
//                 codeword boundary at or after byte sa[i] + P, or its end;
//   item (i, k>0) the piece from byte sa[i] + P k: a speculative entry
//                 (warm-up from SUB_OV bytes early to the first boundary >=
//                 the piece start), then on to the first boundary >= piece
//                 start + P, or the string end.
// A wave takes 64 consecutive items per round (one per lane); their input
// bytes are contiguous (<= 64 P + warm-up) and are staged once in the
// wave's LDS region (coalesced 16-byte loads, byte-swapped to big-endian
// words).  An item's entry is verified against the previous lane's exit (or
// the carry from the previous round); mismatches are re-decoded from the
// settled exit, which makes the result exact for any input.  k = 0 items
// write in pass 1; k > 0 items write in pass 2 at their string's running
// symbol count (a segmented scan across lanes).
// ---------------------------------------------------------------------------
#define WAVE 64
#define DEC_WAVES 16  // waves per decode workgroup: one 64 KB lookup per CU
#define DEC_NT (WAVE * DEC_WAVES)
#define TASK_STR 64                                // strings per wave task
#define PIECE_BYTES 64u                            // input bytes per item (string piece)
#define SUB_OV 24u                                 // warm-up bytes of a k > 0 piece
#define IBUF_W (PIECE_BYTES * WAVE + SUB_OV + 80u)  // per-wave staged input (+ warm-up, alignment, reach)
#define XFAIL 0xFFFFFFFFu    // exit after EOS (sticky failure)
#define XUNKNOWN 0xFFFFFFFEu // speculative entry lost (EOS during warm-up)
#define NOSPEC 0xFFFFFFFDu   // lane has no speculative item

struct SubOut {
  uint32_t entry, exit, cnt;
  uint32_t t, win;  // when the decode reached the string end: tail bits, last window
  bool at_end;
};

// 32-bit window at bit bp >= 1 of the staged round (big-endian words):
// with k = (bp - 1) >> 5 the window starts sh = bp - 32 k in [1, 32] bits into
// {w[k], w[k+1]}, i.e. it is ({w[k], w[k+1]} >> (32 - sh))[31:0] -- one
// v_alignbit on the ds_read2 pair, shift (32 - sh) & 31 = ~(bp - 1) & 31.
__device__ __forceinline__ uint32_t win_q(const lds_u32 *ibe, uint32_t q) {  // q = bp - 1
  const uint32_t k = q >> 5;
  return __builtin_amdgcn_alignbit(ibe[k], ibe[k + 1], ~q);
}
__device__ __forceinline__ uint32_t win_at(const lds_u32 *ibe, uint32_t bp) { return win_q(ibe, bp - 1u); }

// Decode output sinks.  put(v, c8) appends c8 / 8 (1..2) symbols: sym1 in
// bits 0..7 of v, sym2 in bits 8..15 (zero when c8 = 8).
struct NullSink {
  uint32_t n8 = 0;
  __device__ __forceinline__ uint32_t count() const { return n8 >> 3; }
  __device__ __forceinline__ void put(uint32_t, uint32_t c8) { n8 += c8; }
  __device__ __forceinline__ void put_nf(uint32_t, uint32_t c8) { n8 += c8; }
  __device__ __forceinline__ void put2(uint32_t e1, uint32_t e2) { n8 += E_CNT8(e1) + E_CNT8(e2); }
  __device__ __forceinline__ void flush() {}
};
// Caller slots (any alignment, capacity checked), straight to global memory:
// the head dword (which may hold the previous piece's bytes) bytewise, every
// later complete dword whole, every store limited to the slot end `lim`; a
// byte at or past it is not written and marks the overflow.
struct CheckedDwordSink {
  uint32_t *p;
  const uint8_t *lim;
  uint64_t acc;
  uint32_t nb, n8, h;
  bool ovf;
  __device__ __forceinline__ void init(uint8_t *q, uint32_t cap) {
    h = (uint32_t)(uintptr_t)q & 3u;
    p = reinterpret_cast<uint32_t *>(q - h);
    lim = q + cap;
    acc = 0;
    nb = 8u * h;
    n8 = 0;
    ovf = false;
  }
  __device__ __forceinline__ uint32_t count() const { return n8 >> 3; }
  __device__ __forceinline__ void put_nf(uint32_t v, uint32_t c8) {
    // the entry's bytes 0 and 2 as a contiguous pair (byte 1, 3: zero)
    acc |= (uint64_t)__builtin_amdgcn_perm(0u, v, 0x0C0C0200u) << nb;
    nb += c8;
    n8 += c8;
  }
  __device__ __forceinline__ void put(uint32_t v, uint32_t c8) {
    put_nf(v, c8);
    flush();
  }
  __device__ __forceinline__ void bytes(uint32_t from, uint32_t to) {
    uint8_t *b = reinterpret_cast<uint8_t *>(p);
    for (uint32_t x = from; x < to; ++x) {
      if (b + x < lim) b[x] = (uint8_t)(acc >> (8u * x));
      else ovf = true;
    }
  }
  __device__ __forceinline__ void flush() {
    if (nb >= 32u) {
      if (h == 0 && reinterpret_cast<const uint8_t *>(p) + 4 <= lim) *p = (uint32_t)acc;
      else bytes(h, 4u);
      h = 0;
      ++p;
      acc >>= 32;
      nb -= 32u;
    }
  }
  __device__ __forceinline__ void finish() {
    const uint32_t na = nb >> 3;
    if (na > h) bytes(h, na);
  }
};

// Code longer than the lookup: one read of the leading-ones table.  Every
// HPACK code past 13 bits starts with n1 >= 12 ones, a zero and at most 5
// more bits (tools/gen_tables.py long_ones_table), so (n1, those 5 bits)
// names the code.  (Round 5; before: a second-level lookup for 14..16-bit
// codes, then a search over the left-justified limits by leading ones and a
// canonical-symbol read -- up to five dependent LDS reads for a 28-bit code.)
// Returns a lookup-style entry (cnt 1, used = L), or ~0u when EOS (symbol
// 256) completes within `rem`.
__device__ __forceinline__ uint32_t long_index(uint32_t win);
template <class TT>
__device__ __forceinline__ uint32_t long_entry(const TT &T, uint32_t win, uint32_t rem) {
  // (n1 leading ones, clamped to 12..31, then the 5 bits after the first
  // zero: win << (n1 + 1), by alignbit so that n1 = 31 gives 0)
  const uint32_t v = T.long1[long_index(win)];
  const uint32_t L = E_USED(v);
#if DD_SLOWU
  // (selects, not an early return: no exec-mask branch in the slow path)
  const bool fits = L <= rem;
  const uint32_t r = fits ? v & ~E_EOS : v & ~(E_EOS | 0xFFu);
  return fits && (v & E_EOS) ? 0xFFFFFFFFu : r;
#else
  if (L <= rem && (v & E_EOS)) return 0xFFFFFFFFu;
  return L <= rem ? v & ~E_EOS : v & ~(E_EOS | 0xFFu);
#endif
}
// The index of a window's code in T.long1 (long_entry's read).
__device__ __forceinline__ uint32_t long_index(uint32_t win) {
  const uint32_t n1 = min(max((uint32_t)__clz((int)~win), (uint32_t)HD_HUFF_LONG1_N0),
                          (uint32_t)(HD_HUFF_LONG1_N0 + HD_HUFF_LONG1_ROWS - 1));
  return (n1 - HD_HUFF_LONG1_N0) * 32u + (__builtin_amdgcn_alignbit(win, 0u, 31u - n1) >> 27);
}

// First-level miss: the code is longer than the lookup.
template <class TT>
__device__ __forceinline__ uint32_t slow_entry(const TT &T, uint32_t win, uint32_t rem) {
  return long_entry(T, win, rem);
}

// Decode from bit bp (positions relative to the staged round) of a string
// ending at bit bend.  SPEC: warm up to the first boundary >= bseg (the
// entry).  Then decode, emitting into sink, to the first boundary >= bstop,
// or to the string end (tail analysis).  While >= 30 bits remain and the
// step cannot cross bstop, the loop carries no end checks; the rest goes
// through a checked loop.  Window bits past bend are don't-care: a code is
// taken only if it ends at or before bend.
template <bool SPEC, class Sink>
__device__ __forceinline__ SubOut decode_item(const DecTables &T, const lds_u32 *ibe, uint32_t bp,
                                              uint32_t bseg, uint32_t bstop, uint32_t bend,
                                              Sink &sink) {
  SubOut r;
  r.cnt = 0;
  r.t = 0;
  r.win = 0;
  r.at_end = false;
  if (SPEC) {
    while (bp < bseg) {
      const uint32_t w = win_at(ibe, bp);
      const uint32_t rem = bend - bp;
      uint32_t e = T.lut[w >> (32 - HD_HUFF_LUT_BITS)];
      if (e == 0u) e = slow_entry(T, w, rem);
      if (e == 0xFFFFFFFFu) {
        r.entry = r.exit = XUNKNOWN;
        return r;
      }
      const uint32_t L1 = E_L1(e), U = E_USED(e);
      if (L1 > rem) break;  // reached the string's tail
      const bool two = E_CNT(e) == 2u && bp + L1 < bseg && U <= rem;
      bp += two ? U : L1;
    }
  }
  r.entry = bp;
  const uint32_t c0 = sink.count();
  // fast: 2-symbol steps while bp + 12 < bstop and bp + 30 <= bend, in pairs
  // (one bound check and one sink flush per pair) while a whole pair fits,
  // then single steps.  One loop exit: EOS (the FSM's sticky failure state)
  // drops the bounds; a step at the EOS position emits nothing and does not
  // move, so the rest of its pair is idempotent.
  int32_t F = min((int32_t)bstop - 13, (int32_t)bend - 30);  // bound for q = bp - 1
  int32_t F2 = F - 30;  // a first step consumes <= 30 bits
  uint32_t q = bp - 1u;
#define DEC_FAST_STEP()                                          \
  do {                                                           \
    const uint32_t w = win_q(ibe, q);                            \
    uint32_t e = T.lut[w >> (32 - HD_HUFF_LUT_BITS)];            \
    if (e == 0u) {                                               \
      e = slow_entry(T, w, 30u);                                 \
      if (e == 0xFFFFFFFFu) {                                    \
        F = F2 = INT32_MIN;                                      \
        e = 0u;                                                  \
      }                                                          \
    }                                                            \
    sink.put_nf(e & E_OUT2, E_CNT8(e));                          \
    q += E_USED(e);                                              \
  } while (0)
  while ((int32_t)q < F2) {
    DEC_FAST_STEP();
    DEC_FAST_STEP();
    sink.flush();
  }
  while ((int32_t)q < F) {
    DEC_FAST_STEP();
    sink.flush();
  }
#undef DEC_FAST_STEP
  bp = q + 1u;
  bool failed = F == INT32_MIN;
  // checked: to the first boundary >= bstop, or the string's tail
  while (!failed && bp < bstop) {
    const uint32_t rem = bend - bp;
    if (rem == 0) break;
    const uint32_t w = win_at(ibe, bp);
    uint32_t e = T.lut[w >> (32 - HD_HUFF_LUT_BITS)];
    if (e == 0u) {
      e = slow_entry(T, w, rem);
      if (e == 0xFFFFFFFFu) {
        failed = true;
        break;
      }
    }
    const uint32_t L1 = E_L1(e), U = E_USED(e);
    if (L1 > rem) {  // the tail is a proper prefix of a code
      r.at_end = true;
      r.t = rem;
      r.win = w;
      break;
    }
    const bool two = E_CNT(e) == 2u && U <= rem && bp + L1 < bstop;
    sink.put(two ? e & E_OUT2 : e & E_OUT1, two ? 16u : 8u);
    bp += two ? U : L1;
  }
  if (!failed && bp == bend) r.at_end = true;
  r.exit = failed ? XFAIL : bp;
  r.cnt = sink.count() - c0;
  return r;
}

// Final reference decode context and status of a string from the decode of
// its last item (lib/nghttp2_hd_huffman.c:135-142).  The tail is the last
// t < 30 bits: a proper prefix of a code, i.e. an internal node of the code
// tree -> the FSM state it leaves behind (DESIGN.md "decode state").
__device__ __forceinline__ int32_t finish_string(const DecTables &T, const SubOut &r, uint32_t nsym,
                                                 bool ovf, uint32_t *fs, uint32_t *fl) {
  if (r.exit == XFAIL || r.entry == XFAIL) {
    *fs = FAIL_STATE;
    *fl = 0;
    return ovf ? NGHTTP2_AMD_ERR_BUFFER_ERROR : NGHTTP2_AMD_ERR_HEADER_COMP;
  }
  const uint32_t t = r.t;
  const uint32_t v = t ? (r.win >> (32 - t)) : 0u;
  const bool accept = (t <= 7) && (v == (1u << t) - 1u);
  *fs = t ? T.depth_ids[T.depth_base[t] + (v - T.depth_lo[t])] : 0u;
  *fl = (accept ? HUFF_ACCEPTED : 0u) | ((t < 4 && nsym) ? HUFF_SYM : 0u);
  if (ovf) return NGHTTP2_AMD_ERR_BUFFER_ERROR;
  return accept ? (int32_t)nsym : NGHTTP2_AMD_ERR_HEADER_COMP;
}

// Engine slot layout (AUTO): slot_s = 4 * (ceil(floor(8 x_s / 5) / 4) + s)
// with x_s = off[s] - off[0].  Every slot is 4-byte aligned and holds at
// least floor(8 E_s / 5) + 1 bytes (the reference's allocation,
// lib/nghttp2_hd.c:2080-2082) rounded up to a whole dword.
__device__ __host__ __forceinline__ uint64_t auto_slot(uint32_t x, uint32_t s) {
  const uint64_t g = ((uint64_t)x * 8u) / 5u;
  return 4u * (((g + 3u) >> 2) + s);
}

// One lane's item within its wave's round (positions relative to the
// wave's staged input).
struct ItemPos {
  uint32_t i, k;        // task string, piece
  uint32_t a, b, s;     // string bytes [a, b), piece start s
  bool last;            // the string's last piece
};

// Wave tasks: a wave owns TASK_STR consecutive strings at a time and runs
// its own rounds of 64 items (one per lane) over them -- no workgroup
// barriers, so staging, decoding and the bookkeeping of different waves
// overlap freely.  Verify and the segmented scan are wave-level (shuffles).
// Output: the caller's slots (decode_batch), capacity-checked.
struct DecShared {
  DecTables T;  // first: the lookup sits at LDS offset 0 (its base folds into ds_read's offset)
  uint32_t ibe[DEC_WAVES][IBUF_W / 4 + 4];  // per wave: 16 spare bytes, then the round's input
};

__global__ __launch_bounds__(DEC_NT) void k_decode(const uint8_t *__restrict__ src,
                                                   const uint32_t *__restrict__ off, uint32_t n,
                                                   uint8_t *__restrict__ dst,
                                                   const uint32_t *__restrict__ dst_off,
                                                   int32_t *__restrict__ status,
                                                   uint16_t *__restrict__ fstate_out,
                                                   uint8_t *__restrict__ flags_out) {
  __shared__ DecShared S;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  lds_u32 *ibw = (lds_u32 *)S.ibe[wv];
  const lds_u32 *ibe = ibw;
  stage_dec_tables(S.T, DEC_NT);  // the kernel's only workgroup barrier
  const uint32_t ntask = (n + TASK_STR - 1u) / TASK_STR;
  for (uint32_t task = blockIdx.x * DEC_WAVES + wv; task < ntask; task += gridDim.x * DEC_WAVES) {
    const uint32_t t0 = task * TASK_STR;
    const uint32_t nstr = min(n - t0, (uint32_t)TASK_STR);
    // lane l: task string l
    const bool sl = lane < nstr;
    const uint32_t a_l = sl ? off[t0 + lane] : 0u;
    const uint32_t b_l = sl ? off[t0 + lane + 1] : 0u;
    const uint32_t m_l = sl ? (b_l - a_l > PIECE_BYTES ? (b_l - a_l + PIECE_BYTES - 1u) / PIECE_BYTES : 1u) : 0u;
    const uint32_t P_l = wave_incl_scan(m_l);       // items through string l
    const uint32_t X_l = P_l - m_l;                 // first item of string l
    const uint32_t M = __builtin_amdgcn_readlane(P_l, 63);
    uint32_t carry_exit = 0, carry_cnt = 0, IB_prev = 0;
    for (uint32_t r0 = 0; r0 < M; r0 += WAVE) {
      const uint32_t nv = min(M - r0, (uint32_t)WAVE);  // items this round
      const uint32_t q = r0 + lane;
      const bool valid = lane < nv;
      // ---- this lane's item: string = first i with P_i > q
      ItemPos it;
      {
        uint32_t lo = 0, hi = nstr - 1u;
#pragma unroll
        for (int st = 0; st < 6; ++st) {
          const uint32_t mid = (lo + hi) >> 1;
          const uint32_t pm = __shfl(P_l, mid, 64);
          if (pm > q) hi = mid; else lo = mid + 1u;
        }
        it.i = min(lo, nstr - 1u);
        it.k = q - __shfl(X_l, it.i, 64);
        it.a = __shfl(a_l, it.i, 64);
        it.b = __shfl(b_l, it.i, 64);
        it.s = it.a + PIECE_BYTES * it.k;
        it.last = it.s + PIECE_BYTES >= it.b;
      }
      // ---- stage the round's input: [first item (- warm-up), last item's reach)
      const uint32_t A = __builtin_amdgcn_readlane(it.k ? it.s - SUB_OV : it.s, 0);
      const uint32_t Z = __builtin_amdgcn_readlane(min(it.b, it.s + PIECE_BYTES), nv - 1u) + 12u;
      const uint32_t IB = A & ~15u;
      const uint32_t IBX = IB - 16u;  // bit positions: 8 * (byte - IBX) >= 128
      {
        const uint32_t nchunk = (((Z + 15u) & ~15u) - IB) >> 4;
        const uint4 *g = reinterpret_cast<const uint4 *>(src + IB);
        for (uint32_t c = lane; c < nchunk; c += WAVE) {
          const uint4 v = g[c];
          reinterpret_cast<lds_u32 *>(ibw)[4u * c + 4u] = __builtin_bswap32(v.x);
          reinterpret_cast<lds_u32 *>(ibw)[4u * c + 5u] = __builtin_bswap32(v.y);
          reinterpret_cast<lds_u32 *>(ibw)[4u * c + 6u] = __builtin_bswap32(v.z);
          reinterpret_cast<lds_u32 *>(ibw)[4u * c + 7u] = __builtin_bswap32(v.w);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      // the carried exit is a bit position of the previous round's staging
      if (carry_exit < NOSPEC) carry_exit -= 8u * (IB - IB_prev);
      IB_prev = IB;
      const uint32_t j = t0 + it.i;
      const uint32_t bseg = 8u * (it.s - IBX);
      const uint32_t bend = 8u * (min(it.b, it.s + PIECE_BYTES + 32u) - IBX);
      const uint32_t bstop = it.last ? bend : 8u * (it.s + PIECE_BYTES - IBX);
      uint64_t o = 0;
      uint32_t cap = 0;
      if (valid) {
        o = dst_off[j];
        cap = dst_off[j + 1] - (uint32_t)o;
      }
      // ---- pass 1: k = 0 exact (written); k > 0 speculative count
      SubOut r;
      r.entry = r.exit = XFAIL;
      r.cnt = 0;
      r.t = r.win = 0;
      r.at_end = false;
      if (valid) {
        bool ovf = false;
        if (it.k == 0) {
          CheckedDwordSink sk;
          sk.init(dst + o, cap);
          r = decode_item<false>(S.T, ibe, bseg, bseg, bstop, bend, sk);
          sk.finish();
          ovf = sk.ovf;
          if (it.last) {
            uint32_t fs = 0, fl = 0;
            status[j] = finish_string(S.T, r, r.cnt, ovf, &fs, &fl);
            if (fstate_out) fstate_out[j] = (uint16_t)fs;
            if (flags_out) flags_out[j] = (uint8_t)fl;
          }
        } else {
          NullSink nk;
          r = decode_item<true>(S.T, ibe, bseg - 8u * SUB_OV, bseg, bstop, bend, nk);
        }
      }
      // ---- verify / redo (wave): the entry of item (i, k > 0) must equal
      // the exit of the previous lane's item (i, k - 1), or the carry.  A
      // mismatched item is re-decoded once its predecessor is settled (not
      // itself mismatched in this iteration); lane 0 is always settled.
      for (uint32_t iter = 0; iter <= WAVE; ++iter) {
        const uint32_t up = __shfl_up(r.exit, 1, 64);
        const uint32_t pred = lane ? up : carry_exit;
        const bool mism = valid && it.k > 0 && (r.entry != pred || r.entry == XUNKNOWN);
        const uint64_t bal = __ballot(mism);
        if (bal == 0) break;
        const bool pred_mism = lane && ((bal >> (lane - 1u)) & 1u);
        if (mism && !pred_mism) {
          if (pred == XFAIL || pred == XUNKNOWN) {
            r.entry = r.exit = XFAIL;
            r.cnt = 0;
          } else {
            NullSink nk;
            r = decode_item<false>(S.T, ibe, pred, bseg, bstop, bend, nk);
          }
        }
      }
      // ---- symbols of each string through each item: segmented inclusive
      // scan over lanes, segments headed by k = 0 items; the first segment
      // continues the carry
      const uint32_t v = valid ? r.cnt : 0u;
      uint32_t ps = v;
      int32_t hm = (!valid || it.k == 0) ? (int32_t)lane : -1;
#pragma unroll
      for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t o2 = __shfl_up(ps, d, 64);
        const int32_t oh = __shfl_up(hm, d, 64);
        if (lane >= d) {
          ps += o2;
          hm = max(hm, oh);
        }
      }
      const uint32_t excl_h = __shfl(ps - v, hm >= 0 ? (uint32_t)hm : 0u, 64);
      const uint32_t seg = hm >= 0 ? ps - excl_h : ps + carry_cnt;
      // ---- pass 2: k > 0 exact, at the string's running symbol count
      if (valid && it.k > 0) {
        const uint32_t soff = seg - r.cnt;
        const uint32_t e0 = r.entry;
        SubOut r2;
        r2.entry = r2.exit = XFAIL;
        r2.cnt = 0;
        r2.t = r2.win = 0;
        r2.at_end = false;
        bool ovf = false;
        if (e0 != XFAIL) {
          CheckedDwordSink sk;
          sk.init(dst + o + min(soff, cap), cap > soff ? cap - soff : 0u);
          r2 = decode_item<false>(S.T, ibe, e0, bseg, bstop, bend, sk);
          sk.finish();
          ovf = soff + r2.cnt > cap;  // this piece or an earlier one overflowed
        } else {
          ovf = soff > cap;
        }
        if (it.last) {
          uint32_t fs = 0, fl = 0;
          status[j] = finish_string(S.T, r2, soff + r2.cnt, ovf, &fs, &fl);
          if (fstate_out) fstate_out[j] = (uint16_t)fs;
          if (flags_out) flags_out[j] = (uint8_t)fl;
        }
      }
      // ---- carry the string running into the next round
      carry_exit = __builtin_amdgcn_readlane(r.exit, nv - 1u);
      carry_cnt = __builtin_amdgcn_readlane(seg, nv - 1u);
      // the next round overwrites the staged input
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
}

// ---------------------------------------------------------------------------
// decode_batch_auto: the item decoder and its helpers
// ---------------------------------------------------------------------------
#ifndef DD_OV
#define DD_OV 20u  // warm-up bytes of a later item (round 2, 24: 314.2 vs 306.5 us on config 3;
                   // round 3 with overshooting warm-ups, 16/18/22: 312.4/308.9/304.8 vs 300.8)
#endif
#ifndef DD_TASK_W
#define DD_TASK_W 32u  // a string's weight in bytes when balancing tasks over workgroups
#endif
#define DD_NONE 0xFFFFFFFCu  // a round's carried exit: the last item ended its string
#ifndef DD_IW64
#define DD_IW64 16
#endif
#ifndef DD_BI64
#define DD_BI64 2304u
#endif
#ifndef DD_BI40
#define DD_BI40 0u
#endif
#ifndef DD_IW40
#define DD_IW40 16
#endif
#ifndef DD_LB40
#define DD_LB40 13  // lookup bits of the long-string instance
#endif
#ifndef DD_LB64
#define DD_LB64 13  // lookup bits of the short-string instance
#endif
#ifndef DD_IP40
#define DD_IP40 40u  // piece bytes of the long-string instance
#endif
#ifndef DD_IP64
// piece bytes of the short-string instance.  Round 6: 96 (was 64): a string
// of 65-96 encoded bytes is one item instead of two, so a task of short
// strings with a few such strings among them needs one budgeted round, not a
// second one for the leftover pieces (config 5, whose adversarial strings
// reach 83 bytes: 98.7 -> 59.9 us; config 2, all <= 64 bytes: 43.6 / 43.7;
// 128: 60.1 / 44.2; profiles/r06/ab/ab_piece96.log)
#define DD_IP64 96u
#endif
#ifndef DD_TS64
#define DD_TS64 64u  // strings per task unit of the 64-byte instance
#endif
#ifndef DD_TK64
#define DD_TK64 1u
#endif
#ifndef DD_TS40
#define DD_TS40 32u  // strings per task unit of the 40-byte instance
#endif
#ifndef DD_TK40
#define DD_TK40 2u  // units per task (the workgroup's last ones: one unit)
#endif
#ifndef DD_TAILU
#define DD_TAILU 2u  // the workgroup's last DD_TAILU x waves units are claimed singly
#endif
#ifndef DD_JIT_TAIL
#define DD_JIT_TAIL 1  // a tail unit is claimed when the wave's task ends, not one task ahead
#endif
#ifndef DD_SK40
#define DD_SK40 2u  // the 40-byte instance serves long codes every 2nd pair (dd_run SLOWK)
#endif
#ifndef DD_DIRECT_MODE
#define DD_DIRECT_MODE 1  // dd_run's direct long codes (SLOWK == 1) when the caller asks: 0 never
#endif
#ifndef DD_DIRECT_MIN
#define DD_DIRECT_MIN 4u  // lanes of a round with long codes that switch the wave's next round to direct
#endif
#ifndef DD_DIRECT_KEEP
#define DD_DIRECT_KEEP 4u  // ... and to keep it on for the round after
#endif
#ifndef DD_DPAIR
#define DD_DPAIR 1  // dd_run: SLOWK 2 as two pairs per loop trip
#endif
#ifndef DD_FSTEP
#define DD_FSTEP 1  // dd_run: fast single steps between the pairs and the careful steps
#endif
#ifndef DD_SLOWU
#define DD_SLOWU 1  // dd_run: the pairs' slow path behind a uniform branch, predicated
#endif
#ifndef DD_SK64
#define DD_SK64 1u  // the 64-byte instance (config 5's 30-bit codes everywhere): every pair
#endif

// Decode symbols into a byte stream in LDS: both bytes of an entry are
// written, the count advances by the entry's symbols.
// k_decode_items sizes for piece bytes IP: the output region of a lane
// (<= (8 IP + 29) / 5 symbols, one byte of slack, dword aligned), the staged
// dwords of a wave, the staged 16-byte chunks per lane
__host__ __device__ constexpr uint32_t di_rb(uint32_t ip) { return (((8u * ip + 29u) / 5u) + 2u + 3u) & ~3u; }
// A round's items span at most `span` input bytes: 64 items of IP bytes, or
// (budgeted rounds, BI > 0) as many of the next 64 items as fit BI bytes.
// Their output regions (di_rb of each item's bytes, laid back to back) then
// take at most 8 BI / 5 + 64 (29 / 5 + 5) bytes.
__host__ __device__ constexpr uint32_t di_span(uint32_t ip, uint32_t bi) { return bi ? bi : WAVE * ip; }
__host__ __device__ constexpr uint32_t di_obb(uint32_t ip, uint32_t bi) {
  return bi ? ((8u * bi) / 5u + 692u + 15u) & ~15u : WAVE * di_rb(ip);
}
__host__ __device__ constexpr uint32_t di_ibw(uint32_t span) {
  return (((span + DD_OV + 64u) / 4u + 8u) + 3u) & ~3u;  // whole 16-byte chunks
}
__host__ __device__ constexpr uint32_t di_pf(uint32_t span) {
  return (span + DD_OV + 8u + 32u + 16u * WAVE - 1u) / (16u * WAVE);
}
template <uint32_t IP, int IW, int LB, uint32_t BI = 0>
struct DIShared {  // k_decode_items
  DecT<LB> T;  // first: the lookup at LDS offset 0
  alignas(16) uint32_t ib[IW][di_ibw(di_span(IP, BI))];
  alignas(16) uint32_t ob[IW][(di_obb(IP, BI) / 4 + 1 + 3) & ~3u];
  uint32_t claimed, claimed1;     // tasks / tail units of the workgroup's range claimed so far
  uint32_t range[2];              // the workgroup's task range (wave 0's search)
  uint8_t tperm[64];              // claim order of the range's tail units (largest first)
  uint32_t tready;                // tperm written (wave 0, after the barrier)
};

struct DiscardSink {  // a warm-up: its symbols belong to the item before
  __device__ __forceinline__ uint32_t count() const { return 0; }
  __device__ __forceinline__ void put_nf(uint32_t, uint32_t) {}
  __device__ __forceinline__ void put2(uint32_t, uint32_t) {}
  __device__ __forceinline__ void put(uint32_t, uint32_t) {}
  __device__ __forceinline__ void flush() {}
};

// The item decoder's sink: a running LDS pointer (one add per step fewer
// than base + count).
struct LdsPtrSink {
  lds_u8 *p, *base;
#if HD_BOUNDS
  lds_u8 *lim;  // the lane's region end
  __device__ __forceinline__ LdsPtrSink(lds_u8 *b, lds_u8 *l) : p(b), base(b), lim(l) {}
#else
  __device__ __forceinline__ LdsPtrSink(lds_u8 *b) : p(b), base(b) {}
#endif
  __device__ __forceinline__ uint32_t count() const { return (uint32_t)(p - base); }
  __device__ __forceinline__ void put_nf(uint32_t v, uint32_t c8) {
    // (round 3: one ds_write_b16 at the byte address -- the LDS runs in
    // unaligned mode, tools/diag/probe -- measured slower: 354.9 vs 296.2 us
    // on config 3, the hardware splits misaligned stores)
#if HD_BOUNDS
    HD_CHECK(p + 2 <= lim, 0x203u);
#endif
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 16);
    p += c8 >> 3;
  }
  __device__ __forceinline__ void put2(uint32_t e1, uint32_t e2) {
    put_nf(e1, E_CNT8(e1));  // (byte stores: no mask)
    put_nf(e2, E_CNT8(e2));
  }
  __device__ __forceinline__ void put(uint32_t v, uint32_t c8) { put_nf(v, c8); }
  __device__ __forceinline__ void flush() {}
};
typedef LdsPtrSink DISink;

// The item decoder's 16-byte input loads (DD_NTL: nontemporal).  Round 5
// made them nontemporal so that the cache kept the next step's raw input --
// a benefit only of a bench that re-encodes the same batch every step.  On
// the round-6 bench, which rotates three distinct batches, plain loads are
// no slower (bench, 100 steps, three alternations: 1966.1 / 1965.3 / 1968.4
// GB/s against 1958.2 / 1957.9 / 1952.7 nontemporal; with one batch 2029.0 /
// 2019.1 / 2033.1 against 2019.2 / 2029.5 / 2029.0), and the 20-byte warm-up
// overlaps of neighbouring rounds are served by the cache again instead of
// HBM (profiles/r06/bench/ntl_*).  (Nontemporal output stores: 0.374 vs
// 0.209 ms.)
#ifndef DD_NTL
#define DD_NTL 0
#endif
__device__ __forceinline__ uint4 dd_ld16(const uint4 *p) {
#if DD_NTL
  const u32x4 v = __builtin_nontemporal_load((const u32x4 *)p);
  return make_uint4(v.x, v.y, v.z, v.w);
#else
  return *p;
#endif
}
__device__ __forceinline__ void dd_st16(uint4 *p, uint4 v) { *p = v; }

// The window of 32 stream bits from bit q + 1 of the staged words (q = bp - 1).
__device__ __forceinline__ uint32_t dd_win(const lds_u32 *ib, uint32_t q) {
  const uint32_t p = q >> 5;
  return __builtin_amdgcn_alignbit(ib[p], ib[p + 1], ~q);
}

// Input word k (big-endian) of a decode: the wave's staged LDS copy.
struct LdsIn {
  const lds_u32 *ib;
#if HD_BOUNDS
  uint32_t nw;  // staged words readable from ib (index -1 is the word before them)
  __device__ __forceinline__ uint32_t operator()(uint32_t k) const {
    HD_CHECK(k + 1u <= nw || k == 0xFFFFFFFFu, 0x202u);
    return ib[k];
  }
#else
  __device__ __forceinline__ uint32_t operator()(uint32_t k) const { return ib[k]; }
#endif
};

struct DDRun {
  bool failed, at_end;
  uint32_t t, win;  // at the string end: tail bits and the last window
};

// Decode from bp (advanced in place) to the first codeword boundary >=
// bstop, or to the string end bend (tail analysis), into sink.
//
// Steps read a register window: A is the staged word holding bit bp - 1, B
// the next, N the one after (prefetched); with nq = ~(bp - 1) the 32 stream
// bits from bp are alignbit(A, B, nq), so a step's only dependent memory
// access is its lookup.  A step or pair advances < 32 bits: at most one word
// boundary, two selects (DD_ADV).  (Round 3: the 64-bit bit buffer this
// replaces, shifted per step and refilled by compare and 64-bit shift, took
// ~6 VALU more per pair: config 3 decode 301.3 vs 295.0 us.)  A fast step
// needs its 14 lookup bits inside the string (bp + 14 <= bend) and must not
// pass the first boundary >= bstop (bp <= bstop - 13: the first symbol of a
// 2-symbol entry is <= 9 bits); pairs run while both steps qualify.  A code
// longer than the lookup (entry 0) stalls the lane for the rest of the pair,
// then goes through slow_entry; one that would pass the string end is its
// tail and leaves the fast loop.  The last bits go through checked steps,
// which also settle the tail: the undecoded t < 30 bits.
#define DD_ADV(U)                                                        \
  do {                                                                   \
    const uint32_t u_ = (U);                                             \
    const bool t_ = u_ > (nq & 31u); /* (bp - 1) & 31 = 31 - (nq & 31) */ \
    nq -= u_;                                                            \
    A = t_ ? B : A;                                                      \
    B = t_ ? N : B;                                                      \
    kw += t_ ? 1 : 0;                                                    \
    N = ib((uint32_t)kw + 2u);                                           \
  } while (0)
// PAIRS: only the fast pairs, none starting past `lim` (no careful steps):
// bp stops at a codeword boundary on the way, for a caller that records it
// and goes on with another dd_run.
template <class Sink, bool SYNC = false, bool PAIRS = false, uint32_t SLOWK = 1, class TT, class IN>
__device__ __forceinline__ DDRun dd_run(const TT &T, const IN &ib, uint32_t &bp,
                                        uint32_t bstop, uint32_t bend, Sink &sink,
                                        int32_t lim = INT32_MAX, bool direct = false,
                                        uint32_t *nslow = nullptr) {
  DDRun r;
  r.at_end = false;
  r.t = 0;
  r.win = 0;
  uint32_t failed = 0;  // (a VGPR flag: a lane-mask bool costs SALU merges every pair)

  // last start of a fast pair: every code it takes starts before bstop (the
  // second step's second symbol at most LB + (LB - 5) bits on) and ends
  // inside the string (two steps take at most 2 LB bits)
  // (SYNC, a warm-up: pairs may pass bstop -- the first boundary at or after
  // it is then one of the last pair's, picked after the loop; the same
  // overshoot for the items' own decode measured slower: 314.5 vs 303.6 us)
  int32_t G2 = min((int32_t)bstop - (SYNC ? 1 : 2 * TT::BITS - 4), (int32_t)bend - 2 * TT::BITS);
  if (PAIRS) G2 = min(G2, lim);
  // (SYNC) the last pair: start (as nq), entries, slow code
  uint32_t pb = ~(bp - 1u), le1 = 0, le2 = 0, ls = 0;
  // (bp = 0: A is the dword before the staged words, never inside a window;
  // an LDS read inside the workgroup's shared struct -- the staged words
  // follow the lookup tables -- so only the LDS reader may come here)
  static_assert(std::is_same<IN, LdsIn>::value, "dd_run reads index -1: LDS-staged input only");
  int32_t kw = (int32_t)(bp - 1u) >> 5;
  uint32_t A = ib((uint32_t)kw), B = ib((uint32_t)kw + 1u), N = ib((uint32_t)kw + 2u);
  uint32_t nq = ~(bp - 1u);
  int32_t nG = ~(G2 - 1);  // bp <= G2  <=>  (int) nq >= ~(G2 - 1)
  // the window words in before the loop (else the loop head waits for every
  // LDS access in flight, the prefetch of N included, each pair)
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  // a code longer than the lookup inside the pair loop: decode it, or leave
  // the pair loop at EOS (failed) or at the string's tail (the careful steps
  // find it again).  Predicated, with `failed` a VGPR flag: the nested
  // branches this replaces left exec-mask merges (≈7 SALU) in every pair,
  // taken or not (round 4: config 3 decode 277.6 -> 258.1 us, config 5
  // 135.1 -> 130.0, config 2 48.8 -> 47.8).  SLOWK > 1: a lane that meets a
  // long code stalls (its entries use no bits and emit nothing) and the
  // long codes are served every SLOWK-th pair, so the wave pays the slow
  // path's dependent reads once for several lanes' codes (config 3, k = 2:
  // 258.1 -> 253.0 us; the 64-byte instance, which serves config 5's 30-bit
  // codes everywhere, keeps k = 1)
#define DD_SLOW()                                                        \
  do {                                                                   \
    const uint32_t rem_ = bend - (~nq + 1u);                             \
    const uint32_t e_ = slow_entry(T, __builtin_amdgcn_alignbit(A, B, nq), rem_); \
    const bool eos_ = e_ == 0xFFFFFFFFu;                                 \
    const bool ok_ = !eos_ && E_L1(e_) <= rem_;                          \
    failed |= eos_ ? 1u : 0u;                                            \
    nG = ok_ ? nG : INT32_MAX;                                           \
    const uint32_t ek_ = ok_ ? e_ : 0u;                                  \
    sink.put(ek_ & E_OUT2, E_CNT8(ek_));                                 \
    const uint32_t U_ = E_USED(ek_);                                     \
    if (SYNC) ls = U_;                                                   \
    DD_ADV(U_);                                                          \
    if (nslow) ++*nslow;                                                 \
  } while (0)
  // The fast pairs run at raised wave priority: the SIMD issues their
  // dependent chain's VALU before other waves' staging, scans and stores
  // (config 3 decode 294.1 vs 297.7 us, config 2 50.6 vs 52.2; priority 3,
  // or priority over the whole run with its careful steps: no better)
  // direct (the 64-byte instance only, SLOWK == 1, chosen per round by the
  // caller: a wave whose last round met many long codes, as config 5's
  // strings of 28- and 30-bit codes do): a window whose first code is past
  // the lookup (e1 = 0) reads that code from the leading-ones table as the
  // pair's second read (its address computed while e1 is in flight), so the
  // pair decodes it instead of stalling for the slow path; a long code that
  // would pass the string end, or EOS, stops the lane for the careful
  // steps.  (Round 5: always on it took config 5 from 103.5 to 94.2 us but
  // config 2, which has no such codes, from 41.6 to 47.4; behind a wave
  // ballot per pair 97.5 / 43.8.  The loop is compiled both ways; the
  // caller switches a wave per round by the count of long codes its lanes
  // met (*nslow: slow-path runs plus direct decodes): sticky per wave,
  // config 2 +0.8 us; per round, on at 4 lanes and kept at 4, config 5
  // 100.9 -> 96.4 with config 2 41.7 -> 41.9, one box, 16 rounds each.)
  uint32_t it = 0, nlong = 0;
  // one fast pair; slow: this pair may serve a long code (the slow path)
  auto pair = [&](auto dir, bool slow) {
    constexpr bool kDirect = decltype(dir)::value;
    {
      const uint32_t w = __builtin_amdgcn_alignbit(A, B, nq);
      const uint32_t e1 = T.lut[w >> (32 - TT::BITS)];
      const uint32_t U1 = E_USED(e1);
      uint32_t e2;
      if (kDirect) {
        const uint32_t li = long_index(w);
        const uint32_t *p2 = e1 ? &T.lut[(w << U1) >> (32 - TT::BITS)] : &T.long1[li];
        e2 = *p2;
        const bool bad = e1 == 0u && ((e2 & E_EOS) || E_USED(e2) > bend - (~nq + 1u));
        e2 = bad ? 0u : e2;
        nG = bad ? INT32_MAX : nG;
        nlong += e1 == 0u ? 1u : 0u;
      } else {
        e2 = T.lut[(w << U1) >> (32 - TT::BITS)];
      }
      sink.put2(e1, e2);
      const uint32_t U2 = E_USED(e2);
      if (SYNC) {
        pb = nq;  // (as bp after the loop)
        le1 = e1;
        le2 = e2;
        ls = 0;
      }
      DD_ADV(U1 + U2);
#if DD_SLOWU
      // (the slow path behind one uniform branch, predicated per lane: the
      // wave takes it whenever one of its lanes met a long code -- on config
      // 3's bytes nearly every serving pair -- and the exec-mask save and
      // restore of a divergent branch cost every time.  Round 6: config 3
      // decode 213.5 / 207.4 vs 216.3 / 210.3 us, configs 2 and 5 -0.7 /
      // -0.3 %, outputs equal; profiles/r06/ab/ab_slow_uniform.log)
      {
        const bool need = slow && e2 == 0u && (!kDirect || e1 != 0u);
        if (__ballot(need)) {
          const uint32_t rem_ = bend - (~nq + 1u);
          const uint32_t e_ = slow_entry(T, __builtin_amdgcn_alignbit(A, B, nq), rem_);
          const bool eos_ = need && e_ == 0xFFFFFFFFu;
          const bool ok_ = need && e_ != 0xFFFFFFFFu && E_L1(e_) <= rem_;
          failed |= eos_ ? 1u : 0u;
          nG = (need && !ok_) ? INT32_MAX : nG;
          const uint32_t ek_ = ok_ ? e_ : 0u;
          sink.put(ek_ & E_OUT2, E_CNT8(ek_));  // (ek_ = 0: two junk bytes, no advance)
          const uint32_t U_ = E_USED(ek_);
          if (SYNC) ls = need ? U_ : ls;
          DD_ADV(U_);
          if (nslow) *nslow += need ? 1u : 0u;
        }
      }
#else
      if (slow && e2 == 0u && (!kDirect || e1 != 0u))
        DD_SLOW(); /* (an e1 of 0 stalls e2 too; direct: e1 = 0 was decoded or stopped) */
#endif
    }
  };
  auto pairs = [&](auto dir) {
    constexpr bool kDirect = decltype(dir)::value;
#if DD_DPAIR
    if constexpr (SLOWK == 2u && !kDirect) {
      // SLOWK 2 as two pairs per trip, the second one serving long codes:
      // the slow-code period is static (no counter parity in SALU) and the
      // loop's exec-mask bookkeeping is paid once per two pairs (round 6:
      // config 3 decode 209.9 / 208.6 / 217.4 vs 213.0 / 210.0 / 220.8 us in
      // three interleaved sets, outputs equal; configs 2 and 5 flat).  A trip
      // starts only where its second pair keeps the single pair's bound (the
      // first takes <= 2 BITS bits and serves no long code); the last pairs,
      // each serving long codes, run one at a time.  (Four pairs per trip,
      // bound 4 BITS + BITS + 30: 216.1 vs 210.0; the SLOWK 1 loop as two
      // pairs, bound BITS + 30: config 2 44.0 vs 42.8, config 5 61.9 vs 60.8
      // -- profiles/r06/ab/ab_pair_trips.log)
      while ((int32_t)nq - (int32_t)(2 * TT::BITS) >= nG) {
        pair(dir, false);
        pair(dir, true);
      }
      while ((int32_t)nq >= nG) pair(dir, true);
      return;
    }
#endif
    while ((int32_t)nq >= nG) {
      ++it;
      pair(dir, SLOWK == 1u || (it & (SLOWK - 1u)) == 0u);
    }
  };
  __builtin_amdgcn_s_setprio(1);
  if (SLOWK == 1u && DD_DIRECT_MODE != 0 && direct) pairs(std::true_type{});
  else pairs(std::false_type{});
  __builtin_amdgcn_s_setprio(0);
  if (nslow) *nslow += nlong;
#undef DD_SLOW
  bp = ~nq + 1u;
  if (SYNC && !failed && (int32_t)bp >= (int32_t)bstop) {
    // the last pair passed bstop: its codeword boundaries in order are the
    // ends of e1's first symbol and of e1, of e2's first symbol and of e2
    // (or of the long code decoded after e1); the entry is the first one at
    // or after bstop (a 1-symbol entry's first end is its end)
    pb = ~pb + 1u;
    const uint32_t c1 = pb + (le1 ? E_L1(le1) : ls), c2 = pb + E_USED(le1);
    const uint32_t c3 = c2 + (le2 ? E_L1(le2) : ls), c4 = c2 + (le2 ? E_USED(le2) : ls);
    bp = c1 >= bstop ? c1 : c2 >= bstop ? c2 : c3 >= bstop ? c3 : c4;
    r.failed = false;
    return r;
  }
  if (PAIRS) {
    sink.flush();
    r.failed = failed;
    return r;
  }
  if (SYNC) {
    // a warm-up only needs the first codeword boundary >= bstop: single
    // steps that take a 2-symbol entry's second symbol only while the first
    // ends before bstop.  EOS, or a code that would pass the string end,
    // leaves the entry unknown (failed; the verify re-decodes the item).
    // (flags as VGPR words, not lane-mask bools, as in the careful steps)
    uint32_t done = (failed || (int32_t)bp >= (int32_t)bstop) ? 1u : 0u;
    while (__ballot(done == 0u)) {
      if (done == 0u) {
        const uint32_t w = __builtin_amdgcn_alignbit(A, B, nq);
        uint32_t e = T.lut[w >> (32 - TT::BITS)];
        if (e == 0u) e = slow_entry(T, w, 30u);
        const uint32_t L1 = E_L1(e), adv = bp + L1 >= bstop ? L1 : E_USED(e);
        const bool bad = e == 0xFFFFFFFFu || bp + adv > bend;
        failed |= bad ? 1u : 0u;
        const uint32_t a = bad ? 0u : adv;
        bp += a;
        DD_ADV(a);
        done = (bad || bp >= bstop) ? 1u : 0u;
      }
    }
    r.failed = failed;
    return r;
  }
  // careful steps: each one predicated on the stop rules instead of branching
  // -- a step takes its first symbol only if the code ends inside the string
  // (L1 <= rem), its second only if that one does too and the first ended
  // before bstop; a first code that does not fit is the string's tail
  // -- with every lane stepping (a finished lane takes nothing): selects
  // instead of exec-mask branches, the rare long code behind one uniform
  // branch
  // (the loop-carried flags are VGPR words: as lane-mask bools every merge
  // of them costs SALU in each step)
#if DD_FSTEP
  // fast single steps first, while one lookup stays inside the string (bp +
  // BITS <= bend) and a 2-symbol entry's second code starts before bstop
  // (its first is <= BITS - 5 bits: bp <= bstop - (BITS - 4)): no stop rules
  // to predicate, a lane leaves on its own (exec mask), a long code is left
  // to the careful steps.  The careful steps then only settle the item's
  // last code or two.  (Round 6: config 3 decode 212.7 / 211.0 vs 214.3 /
  // 212.4 us, config 2 42.3 / 42.5 vs 43.1 / 43.2, config 5 59.7 / 60.2 vs
  // 60.3 / 61.0 in two interleaved sets, outputs equal;
  // profiles/r06/ab/ab_fast_single_steps.log)
  {
    const int32_t S = min((int32_t)bstop - (TT::BITS - 4), (int32_t)bend - TT::BITS);
    int32_t nS = ~(S - 1);  // bp <= S  <=>  (int) nq >= ~(S - 1)
    while (!failed && (int32_t)nq >= nS) {
      const uint32_t w = __builtin_amdgcn_alignbit(A, B, nq);
      const uint32_t e = T.lut[w >> (32 - TT::BITS)];
      nS = e ? nS : INT32_MAX;
      sink.put(e & E_OUT2, E_CNT8(e));  // (e = 0: two junk bytes, no advance)
      DD_ADV(E_USED(e));
    }
    bp = ~nq + 1u;
  }
#endif
  uint32_t done = failed, at_end = 0u, tt = 0u, twin = 0u;
  while (__ballot(done == 0u)) {
    const uint32_t w = __builtin_amdgcn_alignbit(A, B, nq);
    const uint32_t rem = bend - bp;
    const bool stop = done != 0u || bp >= bstop || rem == 0u;
    uint32_t e = T.lut[w >> (32 - TT::BITS)];
    const bool slow = e == 0u && !stop;
    if (__ballot(slow)) {
      if (slow) e = slow_entry(T, w, rem);
    }
    const bool eos = e == 0xFFFFFFFFu && !stop;  // EOS: the sticky failure state
    const uint32_t L1 = E_L1(e), U = E_USED(e);
    const bool take1 = !stop && !eos && L1 <= rem;
    const bool take2 = take1 && E_CNT(e) == 2u && U <= rem && bp + L1 < bstop;
    const bool tail = !stop && !eos && !take1;  // a proper prefix of a code
    at_end |= tail ? 1u : 0u;
    tt = tail ? rem : tt;
    twin = tail ? w : twin;
    const uint32_t adv = take2 ? U : (take1 ? L1 : 0u);
    sink.put(take2 ? (e & E_OUT2) : (take1 ? (e & E_OUT1) : 0u), take2 ? 16u : (take1 ? 8u : 0u));
    bp += adv;
    DD_ADV(adv);
    failed |= eos ? 1u : 0u;
    done |= (eos || !take1 || bp >= bstop) ? 1u : 0u;
  }
  r.at_end = at_end != 0u;
  r.t = tt;
  r.win = twin;
  sink.flush();
  if (!failed && bp == bend) r.at_end = true;
  r.failed = failed;
  return r;
}
#undef DD_ADV

// Status and final decode context of a string (lib/nghttp2_hd_huffman.c:
// 135-142) from its tail: as finish_string, with the FSM state (three table
// reads) only when the caller asked for it.
template <class TT>
__device__ __forceinline__ void dd_finish(const TT &T, bool failed, uint32_t t,
                                          uint32_t win, uint32_t nsym, bool ovf, uint32_t j,
                                          int32_t *status, uint16_t *fstate_out,
                                          uint8_t *flags_out) {
  const uint32_t v = t ? (win >> (32 - t)) : 0u;
  const bool accept = !failed && (t <= 7) && (v == (1u << t) - 1u);
  status[j] = ovf ? NGHTTP2_AMD_ERR_BUFFER_ERROR
                  : (accept ? (int32_t)nsym : NGHTTP2_AMD_ERR_HEADER_COMP);
  if (fstate_out) {
    fstate_out[j] = failed ? (uint16_t)FAIL_STATE
                           : (uint16_t)(t ? T.depth_ids[T.depth_base[t] + (v - T.depth_lo[t])] : 0u);
    flags_out[j] = failed ? 0u
                          : (uint8_t)((accept ? HUFF_ACCEPTED : 0u) | ((t < 4 && nsym) ? HUFF_SYM : 0u));
  }
}


// ---------------------------------------------------------------------------
// Dense decode by items (decode_batch_auto): a string of <= DD_P encoded
// bytes is one item, a longer one is cut into items of DD_P bytes; a wave
// takes 64 consecutive items per round, one per lane, so no lane ever
// crosses a string end.  A string's first item decodes exactly from the
// string start; a later item warms up from DD_OV bytes before its start to
// the first codeword boundary at or after it (verified against the previous
// item's exit, re-decoded on a mismatch).  Symbols go to the lane's LDS
// region; a segmented scan over the items gives each string's symbol count
// (status), a plain scan of the lanes' byte counts places the regions back
// to back from the task's base, and each lane stores its bytes.
// ---------------------------------------------------------------------------
// The claim order of a workgroup range's tail units (k_decode_items, TK > 1):
// largest first by items (ceil(E / IP) per string), so that the units claimed
// last, whose end is the workgroup's, are the short ones.  Wave 0, after the
// workgroup barrier while the other waves decode (before it, every wave
// waited ~5.5 us for it): the range's last DD_TAILU x IW units (<= 64, <= 64
// x TS strings) are read as offsets, their items summed per unit, ranked.
// (r_lo / r_hi in ranges of TK units, as the search returns them.)
template <uint32_t IP, uint32_t TS, uint32_t TK, int IW>
__device__ __forceinline__ void dd_tail_order(const uint32_t *__restrict__ off, uint32_t n,
                                              uint32_t ntask, uint32_t r_lo, uint32_t r_hi,
                                              uint8_t *tperm, uint32_t lane) {
  static_assert(TS == 32u && DD_TAILU * IW <= 64, "tail units: 32 strings, two per 64 lanes");
  const uint32_t u_lo = min(r_lo * TK, ntask), u_hi = min(r_hi * TK, ntask);
  const uint32_t t_mid = max(u_lo, u_hi > u_lo + DD_TAILU * IW
                                       ? u_lo + ((u_hi - u_lo - DD_TAILU * IW) / TK) * TK
                                       : u_lo);
  const uint32_t nt = u_hi - t_mid;  // <= DD_TAILU * IW + TK - 1
  if (nt == 0u) return;
  const uint32_t s0 = t_mid * TS, s1 = min(u_hi * TS, n);
  uint32_t cu = 0;  // lane u: unit u's items
  for (uint32_t j = 0; j < (nt + 1u) / 2u; ++j) {  // units 2j (lanes 0-31), 2j+1 (32-63)
    const uint32_t s = s0 + 64u * j + lane;
    uint32_t it = 0;
    if (s < s1) {
      const uint32_t e = off[s + 1] - off[s];
      it = e > IP ? (e + IP - 1u) / IP : 1u;
    }
    const uint32_t inc = wave_incl_scan(it);
    const uint32_t lo = __builtin_amdgcn_readlane(inc, 31), all = __builtin_amdgcn_readlane(inc, 63);
    cu = lane == 2u * j ? lo : lane == 2u * j + 1u ? all - lo : cu;
  }
  // rank: larger first, ties by index
  uint32_t rank = 0;
  for (uint32_t v = 0; v < nt; ++v) {
    const uint32_t cv = __builtin_amdgcn_readlane(cu, v);
    rank += (cv > cu || (cv == cu && v < lane)) ? 1u : 0u;
  }
  if (lane < nt) tperm[rank] = (uint8_t)lane;
}

template <uint32_t IP, int IW, int LB, uint32_t BI = 0, uint32_t SK = 1, uint32_t TS = TASK_STR,
          uint32_t TK = 1>
__global__ __launch_bounds__(WAVE * IW) void k_decode_items(const uint8_t *__restrict__ src,
                                                        const uint32_t *__restrict__ off,
                                                        uint32_t n, uint8_t *__restrict__ dst,
                                                        uint64_t dst_cap,
                                                        uint32_t *__restrict__ dst_off,
                                                        int32_t *__restrict__ status,
                                                        uint16_t *__restrict__ fstate_out,
                                                        uint8_t *__restrict__ flags_out) {
  __shared__ DIShared<IP, IW, LB, BI> S;
  constexpr uint32_t kSpan = di_span(IP, BI), kPF = di_pf(kSpan);
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  lds_u32 *ibw = (lds_u32 *)S.ib[wv];
  const lds_u32 *ibe = ibw;
  // (budgeted rounds: the lane's output region moves with the round)
  lds_u8 *my_ob = (lds_u8 *)S.ob[wv] + lane * di_rb(IP);
  const lds_u32 *my_ob32 = (const lds_u32 *)my_ob;
  [[maybe_unused]] uint32_t my_rb = di_rb(IP);  // (HD_BOUNDS) the region's bytes
  if (threadIdx.x == 0) {
    S.claimed = 0u;
    S.claimed1 = 0u;
    S.tready = 0u;
  }
  const uint32_t off0 = off[0];
  // units of TS strings; the workgroup ranges are cut in tasks of TK units
  const uint32_t ntask = (n + TS - 1u) / TS;
  const uint32_t nrange = (n + TS * TK - 1u) / (TS * TK);
  // this workgroup's tasks: with 40-byte pieces (long values, whose tasks
  // differ several-fold in work) a contiguous range balanced by weight
  // (encoded bytes + DD_TASK_W per string) over the grid, its waves striding
  // over it (config 3: 348 vs 356 us); else the grid strides over all tasks
  // (the search costs a short batch more than it saves)
  constexpr bool kBal = IP < 64u;
  uint32_t t_lo, t_hi;
  {
    const uint32_t nwg = gridDim.x, g = blockIdx.x;
    const uint64_t wtot = (uint64_t)(off[n] - off0) + (uint64_t)DD_TASK_W * n;
    // smallest t with weight(t) >= target, for two targets at once (the two
    // 64-ary searches' dependent loads in flight together)
    auto first_at2 = [&](uint64_t ta, uint64_t tb, uint32_t &ra, uint32_t &rb) {
      uint32_t lo_a = 0, hi_a = ta ? nrange : 0u;  // weight(lo) < target <= weight(hi)
      uint32_t lo_b = 0, hi_b = tb ? nrange : 0u;
      while (hi_a - lo_a > 1u || hi_b - lo_b > 1u) {
        const uint32_t st_a = (hi_a - lo_a + WAVE - 1u) / WAVE, st_b = (hi_b - lo_b + WAVE - 1u) / WAVE;
        const uint32_t c_a = min(lo_a + (lane + 1u) * st_a, hi_a), c_b = min(lo_b + (lane + 1u) * st_b, hi_b);
        const uint32_t s_a = min(c_a * (TS * TK), n), s_b = min(c_b * (TS * TK), n);
        const uint32_t o_a = off[s_a], o_b = off[s_b];
        const uint64_t w_a = (uint64_t)(o_a - off0) + (uint64_t)DD_TASK_W * s_a;
        const uint64_t w_b = (uint64_t)(o_b - off0) + (uint64_t)DD_TASK_W * s_b;
        if (hi_a - lo_a > 1u) {
          const uint64_t ge = __ballot(w_a >= ta);  // (lane 63 or the clamp reaches hi)
          const uint32_t j = ge ? (uint32_t)__builtin_ctzll(ge) : WAVE - 1u;
          const uint32_t nhi = __builtin_amdgcn_readlane(c_a, j);
          lo_a = j ? __builtin_amdgcn_readlane(c_a, j - 1u) : lo_a;
          hi_a = nhi;
        }
        if (hi_b - lo_b > 1u) {
          const uint64_t ge = __ballot(w_b >= tb);
          const uint32_t j = ge ? (uint32_t)__builtin_ctzll(ge) : WAVE - 1u;
          const uint32_t nhi = __builtin_amdgcn_readlane(c_b, j);
          lo_b = j ? __builtin_amdgcn_readlane(c_b, j - 1u) : lo_b;
          hi_b = nhi;
        }
      }
      ra = hi_a;
      rb = hi_b;
    };
    // contiguous workgroup ranges (by weight or by count); the weight
    // search runs in wave 0 while the other waves stage the tables
    if (kBal) {
      if (wv == 0) {
        first_at2(wtot * g / nwg, g + 1u == nwg ? 0u : wtot * (g + 1u) / nwg, t_lo, t_hi);
        if (g + 1u == nwg) t_hi = nrange;
        if (lane == 0) {
          S.range[0] = t_lo;
          S.range[1] = t_hi;
        }
      }
      stage_dec_tables(S.T, (WAVE * IW), WAVE);  // the kernel's only workgroup barriers
      t_lo = S.range[0];
      t_hi = S.range[1];
      // the tail's claim order: wave 0, after the barrier (the others start
      // decoding); a tail claim waits for it (in practice it is long ready)
      if constexpr (TK > 1u) {
        if (wv == 0) {
          dd_tail_order<IP, TS, TK, IW>(off, n, ntask, t_lo, t_hi, S.tperm, lane);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          if (lane == 0) __hip_atomic_store((uint32_t *)&S.tready, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    } else {
      stage_dec_tables(S.T, (WAVE * IW));
      t_lo = (uint32_t)((uint64_t)nrange * g / nwg);
      t_hi = g + 1u == nwg ? nrange : (uint32_t)((uint64_t)nrange * (g + 1u) / nwg);
    }
    // in units (a range boundary is a task boundary: tasks of TK units stay
    // aligned to TS * TK strings)
    t_lo = min(t_lo * TK, ntask);
    t_hi = min(t_hi * TK, ntask);
  }
  // Tasks are runs of TK units of TS strings, claimed from the workgroup's
  // LDS counters one task ahead (so the waves of a CU finish within a task
  // of each other): whole tasks (aligned to TS * TK strings) from the range's
  // front, and, TK > 1, single units from its last DD_TAILU x IW units, so
  // that the CU's waves finish within a unit, not a whole task, of each other
  // (round 4, config 3 decode -4 %).
  const uint32_t t_mid = TK > 1u ? max(t_lo, t_hi > t_lo + DD_TAILU * IW
                                                  ? t_lo + ((t_hi - t_lo - DD_TAILU * IW) / TK) * TK
                                                  : t_lo)
                                 : t_hi;
  uint32_t next_k = 0;
  // (defer, DD_JIT_TAIL: a claim that finds the range's whole tasks gone
  // returns kDefer and the wave claims its tail unit when its task ends:
  // claimed one task ahead, the tail units were all handed out a task before
  // the workgroup's end, by stale order, and its waves ended ~22 us apart)
  constexpr uint32_t kDefer = 0xFFFFFFFFu;
  auto claim_next = [&](bool defer, bool tail_only = false) -> uint32_t {
    uint32_t t = 0;
    if (lane == 0) {
      const uint32_t v = tail_only ? 0u : atomicAdd((uint32_t *)&S.claimed, 1u);
      t = tail_only ? t_mid : t_lo + TK * v;
      if (TK > 1u && t + TK > t_mid && defer) {
        t = kDefer;
      } else if (TK > 1u && t + TK > t_mid) {
        const uint32_t c = atomicAdd((uint32_t *)&S.claimed1, 1u);
        if (kBal && c < t_hi - t_mid) {
          while (__hip_atomic_load((uint32_t *)&S.tready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
            __builtin_amdgcn_s_sleep(4);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
          t = t_mid + (uint32_t)S.tperm[c];
        } else {
          t = t_mid + c;
        }
      }
    }
    t = __builtin_amdgcn_readfirstlane(t);
    next_k = t < t_hi ? (t < t_mid ? TK : 1u) : 0u;
    return t;
  };
  constexpr bool kJit = TK > 1u && DD_JIT_TAIL != 0;
  // a task's string offsets are loaded one task ahead, and the first round
  // of the next task is staged into registers during the current task's
  // last round (pf), so neither waits at a task start
  uint32_t na_l = 0, nb_l = 0;
  auto load_offs = [&](uint32_t tk, uint32_t kk, uint32_t &xa, uint32_t &xb) {
    const uint32_t u0 = tk * TS;
    const bool in = tk < ntask && lane < min(n - u0, TS * kk);
    xa = in ? off[u0 + lane] : 0u;
    xb = in ? off[u0 + lane + 1] : 0u;
  };
  // the staged range of a round whose items start at byte R0 (a round's
  // items are contiguous in the pool, the next one starting where the last
  // one ends): [IB, IB + 16 nchunk) = [R0 - OV, min(R0 + 64 P, Z) + 8)
  // (clipped to the task [A, Z), aligned)
  auto round_range = [&](uint32_t R0, uint32_t A, uint32_t Z, uint32_t &IBo, uint32_t &nchunk) {
    IBo = (R0 - A > DD_OV ? R0 - DD_OV : A) & ~15u;
    nchunk = (((min(R0 + kSpan, Z) + 8u + 15u) & ~15u) - IBo) >> 4;
  };
  uint4 pf[kPF];
  uint32_t pf_IB = 0xFFFFFFFFu;
  const uint32_t t_first = claim_next(false);
  uint32_t task_k = next_k;
  load_offs(t_first < t_hi ? t_first : ntask, task_k, na_l, nb_l);
  uint32_t next_task = t_hi;
  // direct long codes (the 64-byte instance, see dd_run): on for the wave's
  // next round when DD_DIRECT_MIN of this round's lanes met a code past the
  // lookup (slow-path runs, or direct decodes of such codes; DD_DIRECT_KEEP
  // of them to stay on)
  bool dmode = false;
  uint32_t nslow = 0;
  for (uint32_t task = t_first; task < t_hi;) {
    next_task = claim_next(kJit);
    const uint32_t t0 = task * TS;
    const uint32_t nstr = min(n - t0, TS * task_k);
    const bool sl = lane < nstr;
    const uint32_t a_l = na_l, b_l = nb_l;
    const uint32_t A = __builtin_amdgcn_readfirstlane(a_l);
    const uint32_t Z = __builtin_amdgcn_readlane(b_l, nstr - 1u);
    load_offs(next_task < t_hi ? next_task : ntask, next_k, na_l, nb_l);
    const uint64_t tbase = auto_slot(A - off0, t0);
    const bool task_ovf = auto_slot(Z - off0, t0 + nstr) > dst_cap;
    if (__ballot(sl && (b_l < a_l || a_l < off0))) {
      // offsets out of order (a caller error): the task's strings report
      // INVALID_ARGUMENT and write nothing, instead of a near-endless item walk
      if (sl) {
        status[t0 + lane] = NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
        dst_off[t0 + lane] = (uint32_t)min(tbase, dst_cap);
        if (t0 + lane == n - 1u) dst_off[n] = (uint32_t)min(tbase, dst_cap);
      }
      task = next_task;
      task_k = next_k;
      continue;
    }
    // items: m_l of string l, X_l the first
    const uint32_t m_l = sl ? max(1u, (b_l - a_l + IP - 1u) / IP) : 0u;
    const uint32_t P_l = wave_incl_scan(m_l), X_l = P_l - m_l;
    const uint32_t M = __builtin_amdgcn_readlane(P_l, 63);
    uint32_t carry_exit = DD_NONE, carry_cnt = 0, IB_prev = 0, run = 0;
    uint32_t ost_me = 0;  // string `lane`'s output start (task-relative)
    uint32_t R0 = A;
    for (uint32_t r0 = 0, nv = 0; r0 < M; r0 += nv) {
      nv = min(M - r0, (uint32_t)WAVE);  // (budgeted rounds: cut below)
      const uint32_t q = r0 + lane;
      // this lane's item: its string i = the last one with X_i <= q; every
      // string with an item in the round marks its first one (or item 0 of
      // the round), then a max-scan over the lanes
      // (a task of single-item strings: item = string, no map)
      uint32_t i = lane, k = 0, a = a_l, b = b_l;
      if (M != nstr) {
        // every string with an item in the round marks the lane of its first
        // one (or lane 0); item q's string is the last mark at or below q:
        // the first marked string plus the marks in lanes 1..q (round 5: an
        // OR over the wave instead of an LDS map and a max-scan, which frees
        // the map's 4 KB per workgroup)
        const bool mk = sl && P_l > r0 && X_l < r0 + WAVE;
        const uint32_t pos = X_l > r0 ? X_l - r0 : 0u;
        const uint32_t mlo = wave_or(mk && pos < 32u ? 1u << pos : 0u);
        const uint32_t mhi = wave_or(mk && pos >= 32u ? 1u << (pos - 32u) : 0u);
        const uint64_t heads = ((uint64_t)mhi << 32) | mlo;
        const uint32_t first = (uint32_t)__builtin_ctzll(__ballot(mk));
        const uint32_t c = (uint32_t)__builtin_popcountll(heads & (~0ull >> (63u - lane)));
        i = min(first + c, nstr) - 1u;
        k = q - __shfl(X_l, i, 64);
        a = __shfl(a_l, i, 64);
        b = __shfl(b_l, i, 64);
      } else if (BI && r0) {  // (a budgeted round after the first: item q = string q)
        i = min(q, nstr - 1u);
        a = __shfl(a_l, i, 64);
        b = __shfl(b_l, i, 64);
      }
      const uint32_t s = a + IP * k, e = min(b, s + IP);
      if (BI) {
        // budgeted round: the items of the next 64 that fit BI input bytes
        // (the first always does: IP <= BI), each lane's output region right
        // after the one before (no region crosses the round's di_obb bytes)
        const uint32_t x = lane < nv ? e - s : 0u;
        const uint32_t cx = wave_incl_scan(x);
        nv = (uint32_t)__builtin_popcountll(__ballot(lane < nv && cx <= BI));
        const uint32_t rb = lane < nv ? di_rb(x) : 0u;
        my_ob = (lds_u8 *)S.ob[wv] + (wave_incl_scan(rb) - rb);
        my_rb = rb;
        HD_CHECK(wave_incl_scan(rb) <= di_obb(IP, BI), 0x206u);
        my_ob32 = (const lds_u32 *)my_ob;
      }
      const bool valid = lane < nv;
      const bool last = e == b;
      const bool spec = valid && k > 0;
      // ---- stage [first item (- OV), last item's end + 8)
      uint32_t IB, nchunk;
      round_range(R0, A, Z, IB, nchunk);
      const uint32_t IBX = IB - 16u;
      const LdsIn inp{ibe HD_LIM(di_ibw(kSpan))};
      // the prefetched chunks (pf) into the staging buffer, byte-swapped
      auto stage_pf = [&](uint32_t nch) {
#pragma unroll
        for (uint32_t u = 0; u < kPF; ++u) {
          const uint32_t c = lane + WAVE * u;
          if (c < nch) {
            HD_CHECK(4u * c + 8u <= di_ibw(kSpan), 0x201u);
            u32x4 v;
            v.x = __builtin_bswap32(pf[u].x);
            v.y = __builtin_bswap32(pf[u].y);
            v.z = __builtin_bswap32(pf[u].z);
            v.w = __builtin_bswap32(pf[u].w);
            *(lds_u32x4 *)(ibw + 4u * c + 4u) = v;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      };
      {
        const uint4 *g = reinterpret_cast<const uint4 *>(src + IB);
        if (pf_IB != IB) {  // (not prefetched)
#pragma unroll
          for (uint32_t u = 0; u < kPF; ++u)
            if (lane + WAVE * u < nchunk) pf[u] = dd_ld16(g + lane + WAVE * u);
        }
        stage_pf(nchunk);
        // prefetch the next round: of this task, else the next task's first
        pf_IB = 0xFFFFFFFFu;
        uint32_t IBn = 0, ncn = 0;
        if (r0 + nv < M) {
          round_range(__builtin_amdgcn_readlane(e, nv - 1u), A, Z, IBn, ncn);
          pf_IB = IBn;
        } else if (next_task < t_hi) {
          const uint32_t An = __builtin_amdgcn_readfirstlane(na_l);
          const uint32_t Zn = __builtin_amdgcn_readlane(
              nb_l, min(n - next_task * TS, TS * next_k) - 1u);
          round_range(An, An, Zn, IBn, ncn);
          pf_IB = IBn;
        }
        if (pf_IB != 0xFFFFFFFFu) {
          const uint4 *gn = reinterpret_cast<const uint4 *>(src + IBn);
#pragma unroll
          for (uint32_t u = 0; u < kPF; ++u)
            if (lane + WAVE * u < ncn) pf[u] = dd_ld16(gn + lane + WAVE * u);
        }
      }
      if (carry_exit < DD_NONE) carry_exit -= 8u * (IB - IB_prev);
      IB_prev = IB;
      const uint32_t bs = 8u * (s - IBX);
      const uint32_t bend = 8u * (min(b, e + 8u) - IBX);
      const uint32_t bstop = last ? bend : 8u * (e - IBX);
      DISink sk(my_ob HD_LIM(my_ob + my_rb));
      // ---- warm-up of the later items: to the first boundary >= 8 s
      uint32_t entry = bs;
      bool dead = false;  // EOS during the warm-up: entry unknown (re-decoded)
      if (spec) {
        uint32_t bp = 8u * (s - DD_OV - IBX);
        DiscardSink dk;
        const DDRun rw = dd_run<DiscardSink, true, false, SK>(S.T, inp, bp, bs, bend, dk, INT32_MAX,
                                                              dmode, &nslow);
        entry = bp;
        dead = rw.failed;
      }
      // ---- the item's symbols
      uint32_t bp = entry;
      DDRun rr;
      rr.failed = rr.at_end = false;
      rr.t = rr.win = 0;
      // (kMerge: the item is decoded in the verify loop's first pass, by the
      // same inlined decoder as its re-decodes)
      constexpr bool kMerge = BI == 0;
      if (valid && !dead && !kMerge)
        rr = dd_run<DISink, false, false, SK>(S.T, inp, bp, bstop, bend, sk, INT32_MAX, dmode, &nslow);
      uint32_t my_exit = rr.failed ? XFAIL : bp;
      uint32_t my_entry = dead ? XUNKNOWN : entry;
      uint32_t c0 = sk.count();
      // ---- verify the later items against the previous item's exit
      // (kMerge: one inlined decoder for the item and its re-decodes -- a
      // pass decodes the lanes marked run_ from `start`, then verifies)
      bool run_ = kMerge && valid && !dead;
      uint32_t start = entry;
      for (uint32_t iter = 0; iter <= WAVE + (kMerge ? 1u : 0u); ++iter) {
        if (kMerge && __ballot(run_)) {
          if (run_) {
            DISink s3(my_ob HD_LIM(my_ob + my_rb));
            uint32_t bq = start;
            rr = dd_run<DISink, false, false, SK>(S.T, inp, bq, bstop, bend, s3, INT32_MAX, dmode, &nslow);
            my_exit = rr.failed ? XFAIL : bq;
            c0 = s3.count();
          }
          run_ = false;
        }
        const uint32_t up = __shfl_up(my_exit, 1, 64);
        const uint32_t pred = lane ? up : carry_exit;
        const bool mism = spec && (my_entry != pred || my_entry == XUNKNOWN);
        const uint64_t bal = __ballot(mism);
        if (bal == 0) break;
        const bool pred_mism = lane && ((bal >> (lane - 1u)) & 1u);
        if (mism && !pred_mism) {
          DISink s3(my_ob HD_LIM(my_ob + my_rb));
          if (pred == XFAIL || pred == XUNKNOWN || pred == DD_NONE) {
            rr.failed = true;  // the string failed in an earlier item
            rr.at_end = false;
            rr.t = rr.win = 0;
            my_exit = XFAIL;
            c0 = 0u;
          } else if (kMerge) {
            start = pred;  // (re-decoded in the next pass)
            run_ = true;
          } else {
            uint32_t bq = pred;
            rr = dd_run<DISink, false, false, SK>(S.T, inp, bq, bstop, bend, s3, INT32_MAX, dmode, &nslow);
            my_exit = rr.failed ? XFAIL : bq;
            c0 = s3.count();
          }
          my_entry = pred;
        }
      }
      if (SK == 1u && DD_DIRECT_MODE != 0) {
        dmode = __builtin_popcountll(__ballot(nslow != 0u)) >=
                (dmode ? DD_DIRECT_KEEP : DD_DIRECT_MIN);
        nslow = 0;
      }
      // ---- string symbol counts: segmented scan (heads: first items)
      // (the plain inclusive scan of the lanes' byte counts, less its value
      // before the lane's last head; no head yet: plus the carried count)
      const uint32_t V = valid ? c0 : 0u;
      const uint32_t Tinc = wave_incl_scan(V);
      const uint32_t h1 = wave_incl_max((!valid || k == 0) ? lane + 1u : 0u);
      const uint32_t excl_h = __shfl(Tinc - V, h1 ? h1 - 1u : 0u, 64);
      const uint32_t seg = h1 ? Tinc - excl_h : Tinc + carry_cnt;  // inclusive
      HD_CHECK(!valid || V <= my_rb, 0x204u);
      HD_CHECK(!(valid && last) || t0 + i < n, 0x205u);
      if (valid && last)
        dd_finish(S.T, rr.failed, rr.t, rr.win, seg,
                  task_ovf && auto_slot(b - off0, t0 + i + 1u) > dst_cap, t0 + i, status,
                  fstate_out, flags_out);
      // ---- dense placement; a string whose first item is in the round
      // takes its output start from that item's lane
      const uint32_t O_l = run + Tinc - V;
      {
        const uint32_t fq = X_l - r0;  // (wraps for strings that started earlier)
        const uint32_t got = __shfl(O_l, fq & 63u, 64);
        if (sl && X_l >= r0 && fq < nv) ost_me = got;
      }
      // ---- store: each lane stores its region straight to its output bytes
      // with unaligned stores (gfx950 global memory takes them whole):
      // 16-byte pieces, then the tail as 8-, 4-, 2- and 1-byte pieces.
      // (Round 4; before, the regions were realigned to dwords by
      // alignbyte with bytewise heads and tails, or for 64-byte items
      // compacted in LDS and stored 16 bytes per lane: config 3 decode
      // 249.6 -> 238.9 us, config 2 48.0 -> 43.3, config 5 130.4 -> 124.5.)
      {
        const uint64_t g0 = tbase + O_l;
        const bool fits = g0 + V <= dst_cap;
        const uint32_t n16 = fits ? V >> 4 : 0u;
        const uint32_t mx = __builtin_amdgcn_readlane(wave_incl_max(n16), 63);
        uint8_t *o = dst + g0;
#pragma unroll
        for (uint32_t m = 0; m < (di_rb(IP) + 15u) / 16u; ++m) {
          if (m >= mx) break;
          if (m < n16) {
            u32x4 v;
            v.x = my_ob32[4u * m];
            v.y = my_ob32[4u * m + 1u];
            v.z = my_ob32[4u * m + 2u];
            v.w = my_ob32[4u * m + 3u];
            *(u32x4u *)(o + 16u * m) = v;
          }
        }
        if (fits) {
          const uint32_t t = V & 15u;
          uint32_t b = V & ~15u;
          if (t & 8u) {
            *(u32x2u *)(o + b) = u32x2{my_ob32[b >> 2], my_ob32[(b >> 2) + 1u]};
            b += 8u;
          }
          if (t & 4u) {
            *(u32u *)(o + b) = my_ob32[b >> 2];
            b += 4u;
          }
          if (t & 2u) {
            *(u16u *)(o + b) = (uint16_t)(my_ob32[b >> 2] >> (8u * (b & 2u)));
            b += 2u;
          }
          if (t & 1u) o[b] = my_ob[b];
        } else {  // near dst_cap: byte by byte, nothing at or past it
          for (uint32_t x = 0; x < V; ++x)
            if (g0 + x < dst_cap) dst[g0 + x] = my_ob[x];
        }
      }
      run += __builtin_amdgcn_readlane(Tinc, 63);
      R0 = __builtin_amdgcn_readlane(e, nv - 1u);
      carry_exit = __builtin_amdgcn_readlane(last ? DD_NONE : my_exit, nv - 1u);
      carry_cnt = __builtin_amdgcn_readlane(seg, nv - 1u);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    // ---- epilogue: output starts
    if (sl) {
      dst_off[t0 + lane] = (uint32_t)min(tbase + ost_me, dst_cap);
      if (t0 + lane == n - 1u) dst_off[n] = (uint32_t)min(tbase + run, dst_cap);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (kJit && next_task == kDefer) {
      next_task = claim_next(false, true);
      load_offs(next_task < t_hi ? next_task : ntask, next_k, na_l, nb_l);
    }
    task = next_task;
    task_k = next_k;
  }
}

// ---------------------------------------------------------------------------
// decode: the reference's nibble FSM   (lib/nghttp2_hd_huffman.c:111-143)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(WG) void k_decode_fsm(const uint8_t *__restrict__ src,
                                                   const uint32_t *__restrict__ off, uint32_t n,
                                                   uint8_t *__restrict__ dst,
                                                   const uint32_t *__restrict__ dst_off,
                                                   int32_t *__restrict__ status,
                                                   uint16_t *__restrict__ fstate_out,
                                                   uint8_t *__restrict__ flags_out,
                                                   const uint16_t *__restrict__ init_state,
                                                   const uint8_t *__restrict__ init_flags,
                                                   int final) {
  __shared__ uint32_t fsm[257 * 16];
  for (uint32_t i = threadIdx.x; i < 257 * 16; i += WG) fsm[i] = dev::hd_huff_fsm[i];
  __syncthreads();
  for (uint32_t s = blockIdx.x * WG + threadIdx.x; s < n; s += gridDim.x * WG) {
    const uint32_t a = off[s], b = off[s + 1];
    const uint32_t o0 = dst_off[s];
    const uint32_t cap = dst_off[s + 1] - o0;
    ByteOut out;
    out.init(dst + o0);
    uint32_t t = init_state ? (uint32_t)init_state[s] | ((uint32_t)init_flags[s] << 16)
                            : (HUFF_ACCEPTED << 16);
    uint32_t w = 0;
    bool overflow = false;
    for (uint32_t p = a; p < b; p += 4) {
      const uint32_t x = load_be32(src, p, b);
      const uint32_t nbytes = min(4u, b - p);
      for (uint32_t k = 0; k < 2 * nbytes; ++k) {
        t = fsm[(t & 0x1FFu) * 16u + ((x >> (28 - 4 * k)) & 15u)];
        if (t & (HUFF_SYM << 16)) {
          if (w < cap) out.put(t >> 24); else overflow = true;
          ++w;
        }
      }
    }
    out.flush();
    const uint32_t flags = (t >> 16) & 0xFFu;
    int32_t st;
    if (overflow) st = NGHTTP2_AMD_ERR_BUFFER_ERROR;
    else if (final && !(flags & HUFF_ACCEPTED)) st = NGHTTP2_AMD_ERR_HEADER_COMP;
    else st = (int32_t)w;
    status[s] = st;
    if (fstate_out) fstate_out[s] = (uint16_t)(t & 0xFFFFu);
    if (flags_out) flags_out[s] = (uint8_t)flags;
  }
}

#endif  // !HD_PART_ENC
#ifndef HD_PART_DEC
// the measured HBM ceiling (nghttp2_amd_hd__copy_calib): each workgroup
// copies contiguous 16 KB blocks (four coalesced 16-byte loads in flight
// per lane, nontemporal), the grid striding over the blocks
__global__ __launch_bounds__(WG) void k_copy_calib(uint4 *__restrict__ dst,
                                                   const uint4 *__restrict__ src, uint64_t n16) {
  const uint64_t nblk = n16 / (4u * WG);
  for (uint64_t b = blockIdx.x; b < nblk; b += gridDim.x) {
    const uint64_t i = b * 4u * WG + threadIdx.x;
    const u32x4 *s4 = reinterpret_cast<const u32x4 *>(src);
    u32x4 *d4 = reinterpret_cast<u32x4 *>(dst);
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = __builtin_nontemporal_load(s4 + i + k * WG);
#pragma unroll
    for (int k = 0; k < 4; ++k) __builtin_nontemporal_store(v[k], d4 + i + k * WG);
  }
  for (uint64_t i = nblk * 4u * WG + (uint64_t)blockIdx.x * WG + threadIdx.x; i < n16;
       i += (uint64_t)gridDim.x * WG)
    dst[i] = src[i];
}

#endif  // !HD_PART_DEC
// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
[[maybe_unused]] static inline uint32_t ntiles_for(uint32_t n) { return (n + WG - 1) / WG; }
// Persistent grids are sized to what is resident at once (occupancy query
// x CU count, cached per kernel), so no workgroup runs as a second "wave"
// and the LDS tables are staged once per resident workgroup.
template <class K>
static uint32_t resident_blocks(K kernel, int BS, int dev) {
  int cus = NUM_CU, per = DEC_WG_PER_CU;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, BS, 0) != hipSuccess || per < 1)
    per = 1;
  return (uint32_t)(cus * per);
}
// The resident count is cached per kernel and per device (the caller's
// current device): host threads driving different GPUs (or the same one)
// may launch concurrently, so the cache is atomic -- a race only computes
// the same value twice.
#define HD_MAX_DEVICES 64
template <auto KERNEL, int BS, int UNIT = BS>  // UNIT: items per workgroup task
static uint32_t persistent_grid(uint32_t n) {
  static std::atomic<uint32_t> cap[HD_MAX_DEVICES];  // zero-initialised (static storage)
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
  uint32_t c = dev < HD_MAX_DEVICES ? cap[dev].load(std::memory_order_relaxed) : 0u;
  if (c == 0) {
    c = resident_blocks(KERNEL, BS, dev);
    if (dev < HD_MAX_DEVICES) cap[dev].store(c, std::memory_order_relaxed);
  }
  const uint32_t g = (n + UNIT - 1) / UNIT;
  return g < c ? g : c;
}

static int hip_rv(hipError_t e) {
  if (e == hipSuccess) return 0;
  fprintf(stderr, "nghttp2_amd_hd: HIP error %s\n", hipGetErrorString(e));
  return NGHTTP2_AMD_ERR_FATAL;
}

#ifndef HD_PART_ENC
template <uint32_t IP, int IW, int LB, uint32_t BI = 0, uint32_t SK = 1, uint32_t TS = TASK_STR,
          uint32_t TK = 1>
static void launch_decode_items(const uint8_t *src, const uint32_t *src_off, uint32_t n,
                                uint8_t *dst, size_t dst_cap, uint32_t *dst_off,
                                int32_t *status, uint16_t *fstate, uint8_t *flags,
                                hipStream_t st) {
  static_assert(TS >= 1 && TS * TK <= TASK_STR, "a task's strings map to lanes");
  hipLaunchKernelGGL((k_decode_items<IP, IW, LB, BI, SK, TS, TK>),
                     dim3(persistent_grid<k_decode_items<IP, IW, LB, BI, SK, TS, TK>, WAVE * IW, TS * TK * IW>(n)),
                     dim3(WAVE * IW), 0, st, src, src_off, n, dst, (uint64_t)dst_cap, dst_off,
                     status, fstate, flags);
}

// decode_batch_auto's two instances, picked by the batch's mean encoded
// string length enc_bytes / n, so that most strings are one item:
//  - mean <= 48 bytes (header strings): whole 64-byte items in budgeted
//    rounds of at most 2304 input bytes, whose staging and output regions are
//    sized for that budget instead of 64 full items, 16 waves per CU with the
//    13-bit lookup (config 2: 56.0 us, against 71-72 for 64-byte items at 8
//    waves without a budget, 59.7 with a 2048-byte budget, 55.7 / 56.7 with
//    2432 / 2560, 62.8 for the 14-bit lookup at 12 waves; the adversarial
//    config 5: 158.6 us, against 164.3 in 32-byte items);
//  - longer: 40-byte pieces with the 13-bit lookup, whose 32 KB less LDS buys
//    16 waves per CU (config 3: 360 vs 385 us for the 14-bit lookup at 12
//    waves).
// Both write the same layout and are exact for any input; the pick only
// moves time.
static int decode_items(const uint8_t *src, const uint32_t *src_off, uint32_t n, uint64_t enc_bytes,
                        uint8_t *dst, size_t dst_cap, uint32_t *dst_off, int32_t *status,
                        uint16_t *fstate, uint8_t *flags, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!dst_off) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (n == 0) return hip_rv(hipMemsetAsync(dst_off, 0, sizeof(uint32_t), st));
  if (!src || !src_off || !dst || !status) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if ((fstate == nullptr) != (flags == nullptr)) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if ((uint64_t)dst_cap > 0xFFFFFFFFull) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;  // uint32 offsets
  if (enc_bytes <= 48ull * n)
    launch_decode_items<DD_IP64, DD_IW64, DD_LB64, DD_BI64, DD_SK64, DD_TS64, DD_TK64>(src, src_off, n, dst, dst_cap, dst_off, status, fstate, flags, st);
  else
    launch_decode_items<DD_IP40, DD_IW40, DD_LB40, DD_BI40, DD_SK40, DD_TS40, DD_TK40>(src, src_off, n, dst, dst_cap, dst_off, status, fstate, flags, st);
  return hip_rv(hipGetLastError());
}

#endif  // !HD_PART_ENC

#if HD_BOUNDS && !defined(HD_PART_DEC)
// the report's self-test: lane 5 records site 0x1FF
__global__ void k_bounds_selftest() { HD_CHECK(threadIdx.x != 5u, 0x1FFu); }
#endif
// (HD_BOUNDS) this translation unit's first recorded violation site, or 0;
// the words are cleared.  0xFFFFFFFF: the copy failed.
static uint32_t bounds_take_tu() {
#if HD_BOUNDS
  uint32_t w[64];
  if (hipMemcpyFromSymbol(w, HIP_SYMBOL(g_hd_bounds), sizeof(w)) != hipSuccess) return 0xFFFFFFFFu;
  uint32_t site = 0;
  for (uint32_t i = 0; i < 64u; ++i)
    if (!site && w[i]) site = w[i];
  static const uint32_t zero[64] = {};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_hd_bounds), zero, sizeof(zero)) != hipSuccess) return 0xFFFFFFFFu;
  return site;
#else
  return 0u;
#endif
}

extern "C" {
// each translation unit's violation words (HD_BOUNDS), read by
// nghttp2_amd_hd__bounds_check (not exported)
__attribute__((visibility("hidden"))) uint32_t hd_bounds_take_enc(void);
__attribute__((visibility("hidden"))) uint32_t hd_bounds_take_dec(void);

#ifndef HD_PART_DEC
__attribute__((visibility("hidden"))) uint32_t hd_bounds_take_enc(void) { return bounds_take_tu(); }

int nghttp2_amd_hd__bounds_check(uint32_t *site) {
#if HD_BOUNDS
  if (!site) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (*site == 0x5E1F7E57u) hipLaunchKernelGGL(k_bounds_selftest, dim3(1), dim3(64), 0, 0);
  const hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return hip_rv(e);
  const uint32_t a = hd_bounds_take_enc(), b = hd_bounds_take_dec();
  *site = a ? a : b;
  return 0;
#else
  (void)site;
  return 1;  // the product build: no checks compiled in
#endif
}

const char *nghttp2_amd_hd_version(void) { return "nghttp2_amd_hd 0.2.0 gfx950"; }

int nghttp2_amd_hd_huff_tables(void *sym_out, void *dec_out) {
  if (sym_out) {
    uint32_t *o = (uint32_t *)sym_out;
    for (int i = 0; i < 257; ++i) {
      o[2 * i] = host::hd_huff_enc_len[i];
      o[2 * i + 1] = host::hd_huff_enc_code[i];
    }
  }
  if (dec_out) memcpy(dec_out, host::hd_huff_fsm, sizeof(host::hd_huff_fsm));
  return 0;
}

size_t nghttp2_amd_hd_huff_encode_bound(uint64_t raw_bytes, uint32_t n) {
  uint64_t b = (raw_bytes * 30u + 7u) / 8u + (uint64_t)n + 16u;
  return (size_t)((b + 15u) & ~(uint64_t)15u);
}

size_t nghttp2_amd_hd_huff_decode_bound(uint64_t enc_bytes, uint32_t n) {
  uint64_t b = (enc_bytes * 8u) / 5u + 4u * (uint64_t)n + 16u;
  return (size_t)((b + 15u) & ~(uint64_t)15u);
}

// the tile sums, then (8-aligned) their 64-bit prefixes for a large batch
static size_t ws_pre_offset(uint32_t nt) { return (((size_t)nt + 16u) * sizeof(uint32_t) + 7u) & ~(size_t)7u; }
size_t nghttp2_amd_hd_huff_workspace_size(uint32_t n) {
  const uint32_t nt = ntiles_for(n);
  return ws_pre_offset(nt) + (nt > EC_SCAN_TILES ? (size_t)nt * sizeof(uint64_t) : 0u);
}
// k_encode's tile prefixes: scanned in their own launch for a large batch
static const uint64_t *scan_tile_prefix(const uint32_t *tiles, uint32_t nt, void *workspace, hipStream_t st) {
  if (nt <= EC_SCAN_TILES || ((uintptr_t)workspace & 7u)) return nullptr;
  uint64_t *pre = (uint64_t *)((char *)workspace + ws_pre_offset(nt));
  hipLaunchKernelGGL(k_tile_prefix64, dim3(1), dim3(1024), 0, st, tiles, nt, pre);
  return pre;
}

size_t nghttp2_amd_hd_huff_encode_workspace_size(uint64_t raw_bytes, uint32_t n) {
  const size_t slots = raw_bytes / 32u + n + 1u;  // (round-1 per-piece bit counts, 32-byte pieces)
  return nghttp2_amd_hd_huff_workspace_size(n) + ((slots * sizeof(uint16_t) + 15u) & ~(size_t)15u);
}

int nghttp2_amd_hd_huff_encode_count_batch(const uint8_t *src, const uint32_t *src_off,
                                           uint32_t n, uint32_t *enc_len, void *stream) {
  if (n == 0) return 0;
  if (!src || !src_off || !enc_len) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(k_enc_count<false>, dim3(ntiles_for(n)), dim3(EC_CNT_NT), 0, (hipStream_t)stream, src,
                     src_off, n, enc_len, (uint32_t *)nullptr, 0);
  return hip_rv(hipGetLastError());
}

int nghttp2_amd_hd_huff_encode_batch(const uint8_t *src, const uint32_t *src_off,
                                     uint32_t n, uint8_t *dst, size_t dst_cap,
                                     uint32_t *dst_off, void *workspace,
                                     size_t workspace_size, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!dst_off) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (n == 0) return hip_rv(hipMemsetAsync(dst_off, 0, sizeof(uint32_t), st));
  if (!src || !src_off || !dst || !workspace) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (workspace_size < nghttp2_amd_hd_huff_workspace_size(n))
    return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  const uint32_t nt = ntiles_for(n);
  if (nt == 1) {  // one tile: count and pack in one launch
    hipLaunchKernelGGL((k_encode<false, true>), dim3(1), dim3(WG), 0, st, src, src_off, n, dst,
                       (uint64_t)dst_cap, dst_off, (const uint32_t *)nullptr, (const uint64_t *)nullptr);
    return hip_rv(hipGetLastError());
  }
  uint32_t *tiles = (uint32_t *)workspace;
  hipLaunchKernelGGL(k_enc_count<false>, dim3(nt), dim3(EC_CNT_NT), 0, st, src, src_off, n, dst_off, tiles, 1);
  const uint64_t *pre = scan_tile_prefix(tiles, nt, workspace, st);
  hipLaunchKernelGGL(k_encode<false>, dim3(nt), dim3(WG), 0, st, src, src_off, n, dst,
                     (uint64_t)dst_cap, dst_off, (const uint32_t *)tiles, pre);
  return hip_rv(hipGetLastError());
}

size_t nghttp2_amd_hd_emit_strings_bound(uint64_t raw_bytes, uint32_t n) {
  // a 32-bit length takes at most 6 prefix bytes (1 + ceil(32 / 7))
  const uint64_t b = raw_bytes + 6u * (uint64_t)n + 16u;
  return (size_t)((b + 15u) & ~(uint64_t)15u);
}

// workspace: the tile sums of the literal lengths
size_t nghttp2_amd_hd_emit_strings_workspace_size(uint64_t raw_bytes, uint32_t n) {
  (void)raw_bytes;
  return nghttp2_amd_hd_huff_workspace_size(n);
}

// emit_string for a batch in two launches: k_enc_count<true> (code bits per
// string, tile sums of the literal lengths) and k_encode<true> (literal
// offsets, then every literal -- prefix and Huffman or raw payload --
// packed straight into the wire stream)
int nghttp2_amd_hd_emit_strings_batch(const uint8_t *src, const uint32_t *src_off, uint32_t n,
                                      uint64_t raw_bytes, uint8_t *dst, size_t dst_cap,
                                      uint32_t *dst_off, void *workspace, size_t workspace_size,
                                      void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!dst_off) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (n == 0) return hip_rv(hipMemsetAsync(dst_off, 0, sizeof(uint32_t), st));
  if (!src || !src_off || !dst || !workspace) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (workspace_size < nghttp2_amd_hd_emit_strings_workspace_size(raw_bytes, n) ||
      dst_cap < nghttp2_amd_hd_emit_strings_bound(raw_bytes, n))
    return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  const uint32_t nt = ntiles_for(n);
  if (nt == 1) {  // one tile: count and pack in one launch
    hipLaunchKernelGGL((k_encode<true, true>), dim3(1), dim3(WG), 0, st, src, src_off, n, dst,
                       (uint64_t)dst_cap, dst_off, (const uint32_t *)nullptr, (const uint64_t *)nullptr);
    return hip_rv(hipGetLastError());
  }
  uint32_t *tiles = (uint32_t *)workspace;
  hipLaunchKernelGGL(k_enc_count<true>, dim3(nt), dim3(EC_CNT_NT), 0, st, src, src_off, n, dst_off, tiles, 1);
  const uint64_t *pre = scan_tile_prefix(tiles, nt, workspace, st);
  hipLaunchKernelGGL(k_encode<true>, dim3(nt), dim3(WG), 0, st, src, src_off, n, dst,
                     (uint64_t)dst_cap, dst_off, (const uint32_t *)tiles, pre);
  return hip_rv(hipGetLastError());
}

int nghttp2_amd_hd__copy_calib(void *dst, const void *src, size_t bytes, void *stream) {
  if (!dst || !src || ((uintptr_t)dst & 15u) || ((uintptr_t)src & 15u) || (bytes & 63u))
    return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (bytes == 0) return 0;
  hipLaunchKernelGGL(k_copy_calib, dim3(NUM_CU * 8), dim3(WG), 0, (hipStream_t)stream, (uint4 *)dst,
                     (const uint4 *)src, (uint64_t)(bytes / 16u));
  return hip_rv(hipGetLastError());
}

int nghttp2_amd_hd_huff_decode_slots(const uint32_t *src_off, uint32_t n, uint32_t *dst_off,
                                     void *workspace, size_t workspace_size, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!dst_off) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (n == 0) return hip_rv(hipMemsetAsync(dst_off, 0, sizeof(uint32_t), st));
  if (!src_off || !workspace) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (workspace_size < nghttp2_amd_hd_huff_workspace_size(n))
    return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  const uint32_t nt = ntiles_for(n);
  uint32_t *tiles = (uint32_t *)workspace;
  hipLaunchKernelGGL(k_slot_len, dim3(nt), dim3(WG), 0, st, src_off, n, dst_off, tiles);
  hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(SCAN_WG), 0, st, tiles, nt, dst_off + n);
  hipLaunchKernelGGL(k_scan_apply, dim3(nt), dim3(WG), 0, st, dst_off, n,
                     (const uint32_t *)tiles);
  return hip_rv(hipGetLastError());
}

#endif  // !HD_PART_DEC
#ifndef HD_PART_ENC
__attribute__((visibility("hidden"))) uint32_t hd_bounds_take_dec(void) { return bounds_take_tu(); }

int nghttp2_amd_hd_huff_decode_batch(const uint8_t *src, const uint32_t *src_off,
                                     uint32_t n, uint8_t *dst, const uint32_t *dst_off,
                                     int32_t *status, uint16_t *fstate, uint8_t *flags,
                                     void *stream) {
  if (n == 0) return 0;
  if (!src || !src_off || !dst || !dst_off || !status) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(k_decode, dim3(persistent_grid<k_decode, DEC_NT, TASK_STR * DEC_WAVES>(n)),
                     dim3(DEC_NT), 0, (hipStream_t)stream, src, src_off, n, dst, dst_off, status,
                     fstate, flags);
  return hip_rv(hipGetLastError());
}


int nghttp2_amd_hd_huff_decode_batch_auto(const uint8_t *src, const uint32_t *src_off,
                                          uint32_t n, uint64_t enc_bytes, uint8_t *dst,
                                          size_t dst_cap, uint32_t *dst_off, int32_t *status,
                                          uint16_t *fstate, uint8_t *flags, void *stream) {
  return decode_items(src, src_off, n, enc_bytes, dst, dst_cap, dst_off, status, fstate, flags,
                      stream);
}

int nghttp2_amd_hd_huff_decode_fsm_batch(const uint8_t *src, const uint32_t *src_off,
                                         uint32_t n, uint8_t *dst, const uint32_t *dst_off,
                                         int32_t *status, uint16_t *fstate, uint8_t *flags,
                                         const uint16_t *init_fstate,
                                         const uint8_t *init_flags, int final,
                                         void *stream) {
  if (n == 0) return 0;
  if (!src || !src_off || !dst || !dst_off || !status) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if ((init_fstate == nullptr) != (init_flags == nullptr)) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(k_decode_fsm, dim3(persistent_grid<k_decode_fsm, WG>(n)), dim3(WG), 0, (hipStream_t)stream,
                     src, src_off, n, dst, dst_off, status, fstate, flags, init_fstate,
                     init_flags, final);
  return hip_rv(hipGetLastError());
}

#endif  // !HD_PART_ENC
}  // extern "C"
