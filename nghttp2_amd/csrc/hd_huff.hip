// hd_huff.hip -- MI355X (gfx950) HPACK Huffman engine: kernels + C ABI.
//
// Replaces the reference's scalar loops in lib/nghttp2_hd_huffman.c
// (encode_count :34-43, encode :45-104, decode :111-143) for batches of
// independent header strings laid out SoA in HBM (see
// include/nghttp2_amd_hd.h and DESIGN.md).  Integer/table work only (no
// MFMA): HBM-bound streaming with the code tables staged in LDS.
//
// Kernels
//   k_enc_count   one string per lane: E = ceil(sum of code lengths / 8),
//                 plus the per-256-string tile sum for the offset scan
//   k_scan_tiles  exclusive scan of the tile sums (one workgroup)
//   k_encode      tile scan -> encoded offsets, then MSB-first bit packing
//                 into aligned 32-bit words with EOS-prefix (all ones)
//                 padding (lib/nghttp2_hd_huffman.c:57-101)
//   k_decode      persistent workgroups, one string per lane: canonical
//                 decode with a 12-bit / 2-symbol lookup table in LDS and an
//                 unrolled compare ladder for codes > 12 bits; the final
//                 {fstate, flags} of the reference's nibble FSM
//                 (lib/nghttp2_hd_huffman.c:122-136) is rebuilt exactly from
//                 the undecoded tail bits (DESIGN.md "decode state")
//   k_decode_fsm  the reference's nibble FSM itself (257x16 table in LDS),
//                 kept as the exact cross-check path and for chunked calls
//   k_slot_len / k_scan_apply   tight decode slots (floor(8E/5)+1 each)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/nghttp2_amd_hd.h"

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
#define ENC_OBUF 16384  // LDS output staging per encode workgroup (bytes)
#define DEC_WG 512      // decode workgroup: 8 waves share one table copy
#define DEC_OBUF 32768  // LDS output staging per decode workgroup (bytes)
#define DEC_IBUF 20480  // LDS input staging per decode workgroup (bytes)

// Ablation switches (tools/diag builds variants; product uses defaults)
#ifndef HD_DEC_INSTAGE
#define HD_DEC_INSTAGE 1   // stage each decode tile's input bytes in LDS
#endif
#ifndef HD_DEC_SORT
#define HD_DEC_SORT 1      // length-sorted lane assignment inside a tile
#endif
#ifndef HD_DEC_OUTSTAGE
#define HD_DEC_OUTSTAGE 1  // stage the tile's output slots in LDS
#endif
#ifndef HD_DIAG_SKIP_LOOP
#define HD_DIAG_SKIP_LOOP 0  // diagnostic only: no symbol decoding at all
#endif

#define HUFF_ACCEPTED 0x01u
#define HUFF_SYM 0x02u
#define FAIL_STATE 0x100u

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
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
typedef __attribute__((address_space(3))) uint32_t lds_u32;
template <class BP> struct W32Of { typedef uint32_t type; };
template <> struct W32Of<lds_u8 *> { typedef lds_u32 type; };
template <class BP> using W32 = typename W32Of<BP>::type;

// Word writer for encode output: the stream [o, o+E) receives big-endian
// 32-bit groups; with phase = o & 3 fixed, each group completes one aligned
// word (funnel shift with the pending bytes).  The head word that also holds
// the previous string's bytes, and the tail, are written byte by byte.
template <class BP>  // BP: byte pointer (global or LDS address space)
struct WordOut {
  BP base;
  uint32_t q, o, phase, pend;
  __device__ __forceinline__ void init(BP b, uint32_t start) {
    base = b; q = start; o = start; phase = start & 3u; pend = 0;
  }
  __device__ __forceinline__ void put32(uint32_t be) {
    const uint32_t le = __builtin_bswap32(be);
    if (phase == 0) {
      *reinterpret_cast<W32<BP> *>(base + q) = le;
    } else {
      const uint32_t word = pend | (le << (8 * phase));
      const uint32_t wa = q & ~3u;
      if (wa < o) {
        for (uint32_t k = phase; k < 4; ++k) base[wa + k] = (uint8_t)(word >> (8 * k));
      } else {
        *reinterpret_cast<W32<BP> *>(base + wa) = word;
      }
      pend = le >> (8 * (4 - phase));
    }
    q += 4;
  }
  // append the top `nbytes` (0..4) bytes of `be`, then drain everything
  __device__ __forceinline__ void finish(uint32_t be, uint32_t nbytes) {
    if (q > o) {
      const uint32_t wa = q & ~3u;
      for (uint32_t k = 0; k < phase; ++k) base[wa + k] = (uint8_t)(pend >> (8 * k));
    }
    for (uint32_t k = 0; k < nbytes; ++k) base[q + k] = (uint8_t)(be >> (24 - 8 * k));
  }
};

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

// Same from an LDS staging buffer (byte index relative to the buffer, which
// holds at least 8 readable bytes past every index used).
__device__ __forceinline__ uint32_t load_be32_lds(const uint32_t *buf, uint32_t pos) {
  const uint32_t w0 = buf[pos >> 2];
  const uint32_t w1 = buf[(pos >> 2) + 1];
  return __builtin_bswap32(__builtin_amdgcn_alignbyte(w1, w0, pos & 3u));
}

// ---------------------------------------------------------------------------
// encode, pass 1: per-string encoded length  (lib/nghttp2_hd_huffman.c:34-43)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(WG) void k_enc_count(const uint8_t *__restrict__ src,
                                                  const uint32_t *__restrict__ off,
                                                  uint32_t n,
                                                  uint32_t *__restrict__ out_len,
                                                  uint32_t *__restrict__ tile_sums) {
  __shared__ uint8_t lenT[256];
  __shared__ uint32_t red[WG / 64];
  lenT[threadIdx.x] = dev::hd_huff_enc_len[threadIdx.x];
  __syncthreads();
  const uint32_t s = blockIdx.x * WG + threadIdx.x;
  uint32_t e = 0;
  if (s < n) {
    const uint32_t a = off[s], b = off[s + 1];
    uint32_t bits = 0;
    for (uint32_t c = a & ~15u; c < b; c += 16) {
      const uint4 v = *reinterpret_cast<const uint4 *>(src + c);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const uint32_t p = c + j;
        const uint32_t L = lenT[(w[j >> 2] >> (8 * (j & 3))) & 0xFFu];
        bits += (p >= a && p < b) ? L : 0u;
      }
    }
    e = (bits + 7u) >> 3;
    if (out_len) out_len[s] = e;
  }
  if (tile_sums) {
    uint32_t tot;
    block_excl_scan<WG>(e, red, &tot);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
  }
}

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

// ---------------------------------------------------------------------------
// encode, pass 2: bit packing   (lib/nghttp2_hd_huffman.c:45-104)
// ---------------------------------------------------------------------------
// Bit-pack one string [a, b) MSB-first (lib/nghttp2_hd_huffman.c:57-84) into
// out_base[o ..], padding the last byte with the EOS prefix (:95-101).
template <class BP>
__device__ __forceinline__ void encode_one(const uint2 *codeT, const uint8_t *__restrict__ src,
                                           uint32_t a, uint32_t b, BP out_base, uint32_t o) {
  uint64_t acc = 0;  // MSB-aligned pending bits, nb < 32 between bytes
  uint32_t nb = 0;
  WordOut<BP> out;
  out.init(out_base, o);
  for (uint32_t c = a & ~15u; c < b; c += 16) {
    const uint4 v = *reinterpret_cast<const uint4 *>(src + c);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t p = c + j;
      if (p >= a && p < b) {
        const uint2 e = codeT[(w[j >> 2] >> (8 * (j & 3))) & 0xFFu];
        acc |= (uint64_t)e.x << (32 - nb);
        nb += e.y;
        if (nb >= 32) {
          out.put32((uint32_t)(acc >> 32));
          acc <<= 32;
          nb -= 32;
        }
      }
    }
  }
  const uint32_t pad = (8u - (nb & 7u)) & 7u;
  acc |= (~0ull >> nb) & ~(~0ull >> (nb + pad));
  nb += pad;
  out.finish((uint32_t)(acc >> 32), nb >> 3);
}

__global__ __launch_bounds__(WG) void k_encode(const uint8_t *__restrict__ src,
                                               const uint32_t *__restrict__ off, uint32_t n,
                                               uint8_t *__restrict__ dst, uint64_t dst_cap,
                                               uint32_t *__restrict__ dst_off,
                                               const uint32_t *__restrict__ tile_prefix) {
  __shared__ uint2 codeT[256];
  __shared__ uint32_t red[WG / 64];
  __shared__ uint32_t obuf[ENC_OBUF / 4];
  codeT[threadIdx.x] = make_uint2(dev::hd_huff_enc_code[threadIdx.x],
                                  dev::hd_huff_enc_len[threadIdx.x]);
  const uint32_t s = blockIdx.x * WG + threadIdx.x;
  const uint32_t E = (s < n) ? dst_off[s] : 0u;
  uint32_t tot;
  const uint32_t O0 = tile_prefix[blockIdx.x];
  const uint32_t o = O0 + block_excl_scan<WG>(E, red, &tot);
  const uint32_t Oend = O0 + tot;
  const uint32_t base = O0 & ~3u;
  // The tile's output [O0, Oend) is contiguous: stage it in LDS and store it
  // with coalesced dwords (byte stores only for the two edge words shared
  // with the neighbouring tiles).  Uniform across the workgroup.
  const bool staged = (Oend - base) <= ENC_OBUF && (uint64_t)Oend <= dst_cap;
  if (s < n) {
    dst_off[s] = o;
    if (staged) {
      encode_one(codeT, src, off[s], off[s + 1], (lds_u8 *)obuf, o - base);
    } else if ((uint64_t)o + E <= dst_cap) {  // never write past the pool
      encode_one(codeT, src, off[s], off[s + 1], dst, o);
    }
  }
  if (staged) {
    __syncthreads();
    const uint32_t nwords = (Oend - base + 3u) >> 2;
    for (uint32_t i = threadIdx.x; i < nwords; i += WG) {
      const uint32_t ga = base + 4u * i;
      const uint32_t w = obuf[i];
      if (ga >= O0 && ga + 4u <= Oend) {
        *reinterpret_cast<uint32_t *>(dst + ga) = w;
      } else {
        for (uint32_t k = 0; k < 4; ++k) {
          const uint32_t q = ga + k;
          if (q >= O0 && q < Oend) dst[q] = (uint8_t)(w >> (8 * k));
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// decode: canonical multi-symbol decoder
// ---------------------------------------------------------------------------
#define NLONG 14  // code lengths > HD_HUFF_LUT_BITS (13,14,15,19..28,30)

struct DecTables {
  uint32_t lut[1 << HD_HUFF_LUT_BITS];
  uint32_t long_lim[NLONG];    // exclusive left-justified limit (last: ~0)
  uint32_t long_delta[NLONG];  // canonical base - first code (mod 2^32)
  uint32_t long_len[NLONG];
  uint16_t canon[260];
  uint32_t depth_lo[30];
  uint16_t depth_base[30];
  uint8_t depth_ids[256];
};

__device__ __forceinline__ void stage_dec_tables(DecTables &T, uint32_t nthreads) {
  const uint32_t t = threadIdx.x;
  for (uint32_t i = t; i < (1u << HD_HUFF_LUT_BITS); i += nthreads) T.lut[i] = dev::hd_huff_lut[i];
  for (uint32_t i = t; i < 257; i += nthreads) T.canon[i] = dev::hd_huff_canon_sym[i];
  if (t < 30) {
    T.depth_lo[t] = dev::hd_huff_depth_lo[t];
    T.depth_base[t] = dev::hd_huff_depth_base[t];
  }
  if (t < 256) T.depth_ids[t] = dev::hd_huff_depth_ids[t];
  if (t == 0) {
    uint32_t i = 0;
#define HD_LONG_ROW(LEN, LIM, FIRST, BASE)                                    \
    T.long_lim[i] = (LIM) > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)(LIM);   \
    T.long_delta[i] = (uint32_t)(BASE) - (uint32_t)(FIRST);                  \
    T.long_len[i] = (LEN);                                                   \
    ++i;
    HD_HUFF_LONG_CODES(HD_LONG_ROW)
#undef HD_LONG_ROW
  }
  __syncthreads();
}

// Decode output sinks.  put2(e, cnt): append the cnt (1..2) symbol bytes in
// the low 16 bits of e.  Engine-slot sinks write both bytes unconditionally
// (a stray second byte is overwritten by the next symbol; every slot has a
// spare byte past floor(8E/5)) -- no branch, no accumulator.
template <class BP>  // BP: byte pointer (LDS or global)
struct SlotSink {
  BP p;
  bool ovf;
  __device__ __forceinline__ void init(BP q) { p = q; ovf = false; }
  __device__ __forceinline__ void put2(uint32_t e, uint32_t cnt) {
    p[0] = (uint8_t)e;
    p[1] = (uint8_t)(e >> 8);
    p += cnt;
  }
  __device__ __forceinline__ void finish() {}
};

// Caller slots (any alignment, capacity checked): ByteOut-based.
struct CheckedSink {
  ByteOut out;
  uint32_t cap, n;
  bool ovf;
  __device__ __forceinline__ void init(uint8_t *p, uint32_t c) {
    out.init(p); cap = c; n = 0; ovf = false;
  }
  __device__ __forceinline__ void put2(uint32_t e, uint32_t cnt) {
    for (uint32_t i = 0; i < cnt; ++i) {
      if (n < cap) out.put((e >> (8 * i)) & 0xFFu); else ovf = true;
      ++n;
    }
  }
  __device__ __forceinline__ void finish() { out.flush(); }
};

// Input: either the tile's bytes staged in LDS as big-endian dwords (ibe,
// byte index of a = a - ibase), or src in global memory.  The bit position
// is the only loop state: every step reads the 32-bit window at it (two
// dwords + one 64-bit funnel shift) and looks up the 12-bit / 2-symbol
// table.  While >= 30 bits remain no code can run past the string end, so
// the main loop carries no end checks; the last < 30 bits go through a
// checked tail loop.  Window bits past the end are don't-care: a code is
// taken only if it ends at or before the end.
template <bool LDSIN>
__device__ __forceinline__ uint32_t window_at(const uint32_t *ibe, const uint32_t *gw,
                                              uint32_t bp) {
  const uint32_t wi = bp >> 5;
  uint32_t w0, w1;
  if (LDSIN) {
    w0 = ibe[wi];
    w1 = ibe[wi + 1];
  } else {
    w0 = __builtin_bswap32(gw[wi]);
    w1 = __builtin_bswap32(gw[wi + 1]);
  }
  return (uint32_t)((((uint64_t)w0 << 32) | w1) >> (32u - (bp & 31u)));
}

// Code longer than the lookup: canonical length by binary search over the
// left-justified limits, then the symbol.  Returns a lookup-style entry
// (cnt 1, used = L), or ~0u when EOS (symbol 256) completes within `rem`.
__device__ __forceinline__ uint32_t long_entry(const DecTables &T, uint32_t win, uint32_t rem) {
  uint32_t lo = 0, hi = NLONG - 1;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const uint32_t mid = (lo + hi) >> 1;
    if (lo < hi) {
      if (win < T.long_lim[mid]) hi = mid; else lo = mid + 1;
    }
  }
  const uint32_t L = T.long_len[lo];
  uint32_t sym = 0;
  if (L <= rem) {
    sym = T.canon[(win >> (32 - L)) + T.long_delta[lo]];
    if (sym == 256) return 0xFFFFFFFFu;
  }
  return sym | (L << 16) | (1u << 25) | (L << 27);
}

template <bool LDSIN, class Sink>
__device__ __forceinline__ int32_t decode_one(const DecTables &T, const uint8_t *__restrict__ src,
                                              const uint32_t *ibe, uint32_t ibase,
                                              uint32_t a, uint32_t b, Sink &sink,
                                              uint32_t *fs, uint32_t *fl) {
  const uint32_t *gw = nullptr;
  uint32_t bp;  // bit position (LDS: from the staging base; global: from a & ~3)
  if (LDSIN) {
    bp = 8u * (a - ibase);
  } else {
    gw = reinterpret_cast<const uint32_t *>(src + (a & ~3u));
    bp = 8u * (a & 3u);
  }
  const uint32_t bend = bp + 8u * (b - a);
  uint32_t nsym = 0;
  uint32_t win = 0;
  bool failed = false;
  if (HD_DIAG_SKIP_LOOP) bp = bend;
  // main loop: >= 30 bits left, no end checks
  while (bend - bp >= 30u) {
    win = window_at<LDSIN>(ibe, gw, bp);
    uint32_t e = T.lut[win >> (32 - HD_HUFF_LUT_BITS)];
    if ((e & 0xF0000u) == 0) {
      e = long_entry(T, win, 30u);
      if (e == 0xFFFFFFFFu) {  // EOS decoded: the FSM's sticky failure state
        failed = true;
        break;
      }
    }
    const uint32_t cnt = (e >> 25) & 3u;
    sink.put2(e, cnt);
    nsym += cnt;
    bp += e >> 27;
  }
  // tail: < 30 bits left, every code checked against the end
  uint32_t rem = bend - bp;
  while (!failed && rem) {
    win = window_at<LDSIN>(ibe, gw, bp);
    uint32_t e = T.lut[win >> (32 - HD_HUFF_LUT_BITS)];
    if ((e & 0xF0000u) == 0) {
      e = long_entry(T, win, rem);
      if (e == 0xFFFFFFFFu) {
        failed = true;
        break;
      }
    }
    const uint32_t L1 = (e >> 16) & 31u;
    const uint32_t L2 = (e >> 21) & 15u;
    if (L1 > rem) break;  // the tail is a proper prefix of a code
    const bool two = L2 != 0 && L1 + L2 <= rem;
    const uint32_t cnt = two ? 2u : 1u;
    sink.put2(e, cnt);
    nsym += cnt;
    const uint32_t used = two ? L1 + L2 : L1;
    bp += used;
    rem -= used;
  }
  sink.finish();
  if (failed) {
    *fs = FAIL_STATE;
    *fl = 0;
    return sink.ovf ? NGHTTP2_AMD_ERR_BUFFER_ERROR : NGHTTP2_AMD_ERR_HEADER_COMP;
  }
  // tail = the last `rem` (< 30) bits: a proper prefix of a code, i.e. an
  // internal node of the code tree -> the FSM state it leaves behind.  When
  // rem > 0 the loop left right after reading the window at bp.
  const uint32_t t = rem;
  const uint32_t v = t ? (win >> (32 - t)) : 0u;
  const bool accept = (t <= 7) && (v == (1u << t) - 1u);
  *fs = t ? T.depth_ids[T.depth_base[t] + (v - T.depth_lo[t])] : 0u;
  *fl = (accept ? HUFF_ACCEPTED : 0u) | ((t < 4 && nsym) ? HUFF_SYM : 0u);
  if (sink.ovf) return NGHTTP2_AMD_ERR_BUFFER_ERROR;
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

// Length-sorted lane assignment inside a tile of NT strings: a stable
// counting sort of the strings by (bucketed) encoded length, so each wave
// decodes strings of similar length and no lane idles for long while its
// wave's longest string finishes.  Returns the tile-relative string index
// this lane decodes (>= cnt: none).
template <int NT>
__device__ __forceinline__ uint32_t sorted_lane(uint32_t len, bool live, uint32_t *hist,
                                                uint16_t *perm, uint32_t *red) {
  const uint32_t t = threadIdx.x;
  if (t < 256) hist[t] = 0;
  __syncthreads();
  const uint32_t bkt = len < 192u ? len : min(255u, 192u + ((len - 192u) >> 4));
  uint32_t rank = 0;
  if (live) rank = atomicAdd(&hist[bkt], 1u);
  __syncthreads();
  const uint32_t h = (t < 256) ? hist[t] : 0u;
  uint32_t tot;
  const uint32_t start = block_excl_scan<NT>(h, red, &tot);
  if (t < 256) hist[t] = start;
  __syncthreads();
  if (live) perm[hist[bkt] + rank] = (uint16_t)t;
  __syncthreads();
  return (t < tot) ? (uint32_t)perm[t] : 0xFFFFFFFFu;
}

// AUTO: engine-assigned slots (written out to dst_off), the tile's slots
// staged in LDS and stored with coalesced dwords when they fit; else caller
// slots, capacity-checked, written directly.
template <bool AUTO>
__global__ __launch_bounds__(DEC_WG) void k_decode(const uint8_t *__restrict__ src,
                                                   const uint32_t *__restrict__ off, uint32_t n,
                                                   uint8_t *__restrict__ dst, uint64_t dst_cap,
                                                   uint32_t *__restrict__ dst_off,
                                                   int32_t *__restrict__ status,
                                                   uint16_t *__restrict__ fstate_out,
                                                   uint8_t *__restrict__ flags_out) {
  __shared__ DecTables T;
  __shared__ uint32_t obuf[AUTO ? DEC_OBUF / 4 : 1];
  __shared__ uint4 ibuf[DEC_IBUF / 16 + 1];
  __shared__ uint32_t hist[256];
  __shared__ uint16_t perm[DEC_WG];
  __shared__ uint32_t red[DEC_WG / 64];
  stage_dec_tables(T, DEC_WG);
  const uint32_t off0 = off[0];
  for (uint32_t t0 = blockIdx.x * DEC_WG; t0 < n; t0 += gridDim.x * DEC_WG) {
    const uint32_t mine = t0 + threadIdx.x;
    const bool live0 = mine < n;
    const uint32_t len0 = live0 ? off[mine + 1] - off[mine] : 0u;
    const uint32_t r = HD_DEC_SORT ? sorted_lane<DEC_WG>(len0, live0, hist, perm, red)
                                   : (live0 ? threadIdx.x : 0xFFFFFFFFu);
    const uint32_t s = t0 + r;
    const bool live = r != 0xFFFFFFFFu;
    uint32_t fs = 0, fl = 0;
    int32_t st = 0;
    // stage the tile's input bytes in LDS with one bulk coalesced load
    const uint32_t s1 = min(t0 + DEC_WG, n);
    const uint32_t ibase = off[t0] & ~15u;
    const uint32_t nchunk = (off[s1] - ibase + 15u) >> 4;
    const bool in_lds = HD_DEC_INSTAGE && nchunk <= DEC_IBUF / 16;  // uniform
    if (in_lds) {  // big-endian dwords: the decoder's windows need no swaps
      const uint4 *g = reinterpret_cast<const uint4 *>(src + ibase);
      for (uint32_t i = threadIdx.x; i < nchunk; i += DEC_WG) {
        const uint4 v = g[i];
        ibuf[i] = make_uint4(__builtin_bswap32(v.x), __builtin_bswap32(v.y),
                             __builtin_bswap32(v.z), __builtin_bswap32(v.w));
      }
      if (threadIdx.x == 0) ibuf[nchunk] = make_uint4(0, 0, 0, 0);
      __syncthreads();
    }
    const uint32_t *ib = in_lds ? reinterpret_cast<const uint32_t *>(ibuf) : nullptr;
    if (AUTO) {
      const uint64_t lo = auto_slot(off[t0] - off0, t0);
      const uint64_t hi = auto_slot(off[s1] - off0, s1);
      const bool staged = HD_DEC_OUTSTAGE && (hi - lo) <= DEC_OBUF && hi <= dst_cap;  // uniform
      if (live) {
        const uint32_t a = off[s], b = off[s + 1];
        const uint64_t o64 = auto_slot(a - off0, s);
        dst_off[s] = (uint32_t)o64;
        if (s == n - 1) dst_off[n] = (uint32_t)auto_slot(b - off0, n);
        if (staged) {
          SlotSink<lds_u8 *> sink;
          sink.init((lds_u8 *)obuf + (o64 - lo));
          st = ib ? decode_one<true>(T, src, ib, ibase, a, b, sink, &fs, &fl)
                  : decode_one<false>(T, src, ib, ibase, a, b, sink, &fs, &fl);
        } else if (auto_slot(b - off0, s + 1) > dst_cap) {
          st = NGHTTP2_AMD_ERR_BUFFER_ERROR;
        } else {
          SlotSink<uint8_t *> sink;
          sink.init(dst + o64);
          st = ib ? decode_one<true>(T, src, ib, ibase, a, b, sink, &fs, &fl)
                  : decode_one<false>(T, src, ib, ibase, a, b, sink, &fs, &fl);
        }
      }
      if (staged) {
        __syncthreads();
        const uint32_t nwords = (uint32_t)((hi - lo) >> 2);
        uint32_t *g = reinterpret_cast<uint32_t *>(dst + lo);
        for (uint32_t i = threadIdx.x; i < nwords; i += DEC_WG) g[i] = obuf[i];
      }
    } else if (live) {
      const uint32_t a = off[s], b = off[s + 1];
      const uint32_t o = dst_off[s];
      CheckedSink sink;
      sink.init(dst + o, dst_off[s + 1] - o);
      st = ib ? decode_one<true>(T, src, ib, ibase, a, b, sink, &fs, &fl)
                : decode_one<false>(T, src, ib, ibase, a, b, sink, &fs, &fl);
    }
    if (live) {
      status[s] = st;
      if (fstate_out) fstate_out[s] = (uint16_t)fs;
      if (flags_out) flags_out[s] = (uint8_t)fl;
    }
    __syncthreads();  // obuf / hist / perm reuse by the next tile
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

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
static inline uint32_t ntiles_for(uint32_t n) { return (n + WG - 1) / WG; }
// Persistent grids are sized to what is resident at once (occupancy query
// x CU count, cached per kernel), so no workgroup runs as a second "wave"
// and the LDS tables are staged once per resident workgroup.
template <class K>
static uint32_t resident_blocks(K kernel, int BS) {
  int dev = 0, cus = NUM_CU, per = DEC_WG_PER_CU;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, BS, 0) != hipSuccess || per < 1)
    per = 1;
  return (uint32_t)(cus * per);
}
template <auto KERNEL, int BS>
static uint32_t persistent_grid(uint32_t n) {
  static uint32_t cap = 0;  // one per kernel
  if (cap == 0) cap = resident_blocks(KERNEL, BS);
  const uint32_t g = (n + BS - 1) / BS;
  return g < cap ? g : cap;
}

static int hip_rv(hipError_t e) {
  if (e == hipSuccess) return 0;
  fprintf(stderr, "nghttp2_amd_hd: HIP error %s\n", hipGetErrorString(e));
  return NGHTTP2_AMD_ERR_FATAL;
}

extern "C" {

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

size_t nghttp2_amd_hd_huff_workspace_size(uint32_t n) {
  return ((size_t)ntiles_for(n) + 16u) * sizeof(uint32_t);
}

int nghttp2_amd_hd_huff_encode_count_batch(const uint8_t *src, const uint32_t *src_off,
                                           uint32_t n, uint32_t *enc_len, void *stream) {
  if (n == 0) return 0;
  if (!src || !src_off || !enc_len) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(k_enc_count, dim3(ntiles_for(n)), dim3(WG), 0, (hipStream_t)stream, src,
                     src_off, n, enc_len, (uint32_t *)nullptr);
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
  uint32_t *tiles = (uint32_t *)workspace;
  hipLaunchKernelGGL(k_enc_count, dim3(nt), dim3(WG), 0, st, src, src_off, n, dst_off, tiles);
  hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(SCAN_WG), 0, st, tiles, nt, dst_off + n);
  hipLaunchKernelGGL(k_encode, dim3(nt), dim3(WG), 0, st, src, src_off, n, dst,
                     (uint64_t)dst_cap, dst_off, (const uint32_t *)tiles);
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

int nghttp2_amd_hd_huff_decode_batch(const uint8_t *src, const uint32_t *src_off,
                                     uint32_t n, uint8_t *dst, const uint32_t *dst_off,
                                     int32_t *status, uint16_t *fstate, uint8_t *flags,
                                     void *stream) {
  if (n == 0) return 0;
  if (!src || !src_off || !dst || !dst_off || !status) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(k_decode<false>, dim3(persistent_grid<k_decode<false>, DEC_WG>(n)), dim3(DEC_WG), 0,
                     (hipStream_t)stream, src, src_off, n, dst, (uint64_t)0,
                     (uint32_t *)dst_off, status, fstate, flags);
  return hip_rv(hipGetLastError());
}

int nghttp2_amd_hd_huff_decode_batch_auto(const uint8_t *src, const uint32_t *src_off,
                                          uint32_t n, uint8_t *dst, size_t dst_cap,
                                          uint32_t *dst_off, int32_t *status,
                                          uint16_t *fstate, uint8_t *flags, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!dst_off) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (n == 0) return hip_rv(hipMemsetAsync(dst_off, 0, sizeof(uint32_t), st));
  if (!src || !src_off || !dst || !status) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(k_decode<true>, dim3(persistent_grid<k_decode<true>, DEC_WG>(n)), dim3(DEC_WG), 0, st, src, src_off,
                     n, dst, (uint64_t)dst_cap, dst_off, status, fstate, flags);
  return hip_rv(hipGetLastError());
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

}  // extern "C"
