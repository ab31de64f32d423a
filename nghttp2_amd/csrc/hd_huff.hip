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

// Ablation switch (tools/diag builds variants; the product uses the default)
#ifndef HD_DEC_OUTSTAGE
#define HD_DEC_OUTSTAGE 1  // stage the decode tile's output slots in LDS
#endif

#ifndef HD_BITBUF
#define HD_BITBUF 1  // fast loop: register bit buffer (1 LDS round trip per step)
#endif
#ifndef HD_DIAG_STAMPS
#define HD_DIAG_STAMPS 0   // diagnostic build only: per-phase s_memtime sums
#endif
#if HD_DIAG_STAMPS
// [wg][slot]: 0 setup, 1 sort, 2 pass1, 3 verify, 4 scan, 5 pass2, 6 report,
// 7 copy, 8 verify iterations, 9 mismatches, 10 rounds, 11 tiles
__device__ unsigned long long g_stamps[4096][16];
#define STAMP(slot, t0)                                                        \
  do {                                                                         \
    __syncthreads();                                                           \
    const unsigned long long t1_ = __builtin_amdgcn_s_memtime();               \
    if (threadIdx.x == 0) g_stamps[blockIdx.x & 4095][slot] += t1_ - (t0);     \
    (t0) = t1_;                                                                \
  } while (0)
#define COUNT(slot, v) do { if (threadIdx.x == 0) g_stamps[blockIdx.x & 4095][slot] += (v); } while (0)
__device__ uint32_t g_dctr[3];  // per-thread loop trips: fast, checked, warm-up (diag)
#define DCTR(k) (++dctr[k])
#else
#define DCTR(k) do { } while (0)
#define STAMP(slot, t0) do { } while (0)
#define COUNT(slot, v) do { } while (0)
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

#define NLONG_PAD 16  // search width (padding rows repeat the last row)
struct DecTables {
  uint32_t lut[1 << HD_HUFF_LUT_BITS];
  uint32_t long_lim[NLONG_PAD];    // exclusive left-justified limit (last: ~0)
  uint32_t long_delta[NLONG_PAD];  // canonical base - first code (mod 2^32)
  uint32_t long_len[NLONG_PAD];
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
    for (; i < NLONG_PAD; ++i) {
      T.long_lim[i] = 0xFFFFFFFFu;
      T.long_delta[i] = T.long_delta[NLONG - 1];
      T.long_len[i] = T.long_len[NLONG - 1];
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Item decoding (DESIGN.md "decode").  A tile is DEC_NS consecutive strings.
// A string of E encoded bytes is cut into m = max(1, ceil(E / 64)) ITEMS:
//   item (i, 0)   the string from its first bit (exact), up to the first
//                 codeword boundary at or after byte sa[i] + 64, or its end;
//   item (i, k>0) the piece from byte sa[i] + 64 k: a speculative entry
//                 (warm-up from SUB_OV bytes early to the first boundary >=
//                 the piece start), then on to the first boundary >= piece
//                 start + 64, or the string end.
// Rounds take DEC_NT consecutive items; their input bytes are contiguous
// (<= 64 DEC_NT + warm-up) and are staged once in LDS (coalesced 16-byte
// loads, byte-swapped to big-endian words).  Lanes are assigned items sorted
// by length, so a wave's lanes finish together.  An item's entry is verified
// against the previous item's exit (or the carry from the previous round);
// mismatches are re-decoded from the settled exit, which makes the result
// exact for any input.  k = 0 items write in pass 1; k > 0 items write in
// pass 2 at their string's running symbol count (a segmented scan).  Output
// goes into an LDS image of the round's slot range and is stored with
// coalesced 16-byte writes.
// ---------------------------------------------------------------------------
#define DEC_NT 256                                 // lanes per decode workgroup
#define DEC_NS 512                                 // strings per decode tile
#define PIECE_BYTES 64u                            // input bytes per item (string piece)
#define SUB_OV 16u                                 // warm-up bytes of a k > 0 piece
#define IBUF_BYTES (PIECE_BYTES * DEC_NT + 96u)    // + warm-up, alignment, overrun, read-ahead
#define DEC_OBUF 30720u                            // LDS output image per round (>= 8/5 IBUF + 4 DEC_NT)
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

// Decode output sinks.  put2(e, cnt) appends the cnt (1..2) symbols of a
// table entry: sym1 in bits 0..7, sym2 in bits 16..23.
//  LdsFast   second byte stored unconditionally: only for items whose
//            following byte is this lane's own next store, slot slack, or a
//            byte that a later phase (after a barrier) rewrites -- pass 1.
//  LdsSafe   second byte to a private junk dword when cnt == 1 -- pass 2,
//            where the next byte belongs to a concurrently running lane.
//  GlobalOut direct stores (round image too large to stage).
template <bool SAFE>
struct LdsSink {
  lds_u8 *p, *junk;
  __device__ __forceinline__ uint32_t count() const { return (uint32_t)(uintptr_t)p; }
  __device__ __forceinline__ void put2(uint32_t e, uint32_t cnt) {
    p[0] = (uint8_t)e;
    lds_u8 *q = p + 1;
    if (SAFE) q = cnt > 1 ? q : junk;
    q[0] = (uint8_t)(e >> 16);
    p += cnt;
  }
};
struct GlobalSink {
  uint8_t *p;
  __device__ __forceinline__ uint32_t count() const { return (uint32_t)(uintptr_t)p; }
  __device__ __forceinline__ void put2(uint32_t e, uint32_t cnt) {
    p[0] = (uint8_t)e;
    if (cnt > 1) p[1] = (uint8_t)(e >> 16);
    p += cnt;
  }
};
// Direct global output of an item that starts on a dword boundary (an
// engine slot): whole dwords from a 64-bit accumulator.  finish(): the
// string's last item may write its final dword whole (the slot is a dword
// multiple and holds more than the decoded bytes); otherwise the tail goes
// bytewise, since the next piece (another lane) continues in that dword.
struct DwordSink {
  uint32_t *p;
  uint64_t acc;
  uint32_t na, n;
  __device__ __forceinline__ void init(uint8_t *q) {
    p = reinterpret_cast<uint32_t *>(q);
    acc = 0;
    na = n = 0;
  }
  __device__ __forceinline__ uint32_t count() const { return n; }
  __device__ __forceinline__ void put2(uint32_t e, uint32_t cnt) {
    const uint32_t v = (e & 0xFFu) | ((e >> 8) & 0xFF00u);
    acc |= (uint64_t)v << (8u * na);
    na += cnt;
    n += cnt;
    if (na >= 4u) {
      *p++ = (uint32_t)acc;
      acc >>= 32;
      na -= 4u;
    }
  }
  __device__ __forceinline__ void finish(bool whole) {
    if (na == 0) return;
    if (whole) {
      *p = (uint32_t)acc;
    } else {
      uint8_t *b = reinterpret_cast<uint8_t *>(p);
      for (uint32_t x = 0; x < na; ++x) b[x] = (uint8_t)(acc >> (8u * x));
    }
  }
};
struct NullSink {
  uint32_t n = 0;
  __device__ __forceinline__ uint32_t count() const { return n; }
  __device__ __forceinline__ void put2(uint32_t, uint32_t cnt) { n += cnt; }
};
// Caller slots (any alignment, capacity checked).
struct CheckedSink {
  uint8_t *p;
  uint32_t cap, n;
  bool ovf;
  __device__ __forceinline__ void init(uint8_t *q, uint32_t c) { p = q; cap = c; n = 0; ovf = false; }
  __device__ __forceinline__ uint32_t count() const { return n; }
  __device__ __forceinline__ void put2(uint32_t e, uint32_t cnt) {
    if (n < cap) p[n] = (uint8_t)e; else ovf = true;
    if (cnt > 1) {
      if (n + 1 < cap) p[n + 1] = (uint8_t)(e >> 16); else ovf = true;
    }
    n += cnt;
  }
};

// Code longer than the lookup: canonical length by a branch-free search over
// the left-justified limits (one row per code length, padded to 16 rows),
// then the symbol.  Returns a lookup-style entry
// (cnt 1, used = L), or ~0u when EOS (symbol 256) completes within `rem`.
__device__ __forceinline__ uint32_t long_entry(const DecTables &T, uint32_t win, uint32_t rem) {
  uint32_t i = 0;
#pragma unroll
  for (uint32_t step = NLONG_PAD / 2; step; step >>= 1)
    i += (T.long_lim[i + step - 1] <= win) ? step : 0u;
  i = min(i, (uint32_t)NLONG - 1u);  // win == ~0: the 30-bit row
  const uint32_t L = T.long_len[i];
  const uint32_t sym = T.canon[(win >> (32 - L)) + T.long_delta[i]];
  if (L <= rem && sym == 256) return 0xFFFFFFFFu;
  return (L <= rem ? sym : 0u) | (L << 8) | (1u << 24) | (L << 27);
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
                                              Sink &sink, uint32_t *dctr) {
  (void)dctr;
  SubOut r;
  r.cnt = 0;
  r.t = 0;
  r.win = 0;
  r.at_end = false;
  if (SPEC) {
    while (bp < bseg) {
      DCTR(2);
      const uint32_t w = win_at(ibe, bp);
      const uint32_t rem = bend - bp;
      uint32_t e = T.lut[w >> (32 - HD_HUFF_LUT_BITS)];
      if (e == 0u) e = long_entry(T, w, rem);
      if (e == 0xFFFFFFFFu) {
        r.entry = r.exit = XUNKNOWN;
        return r;
      }
      const uint32_t L1 = (e >> 8) & 31u, L2 = (e >> 13) & 7u;
      if (L1 > rem) break;  // reached the string's tail
      const bool two = L2 != 0 && bp + L1 < bseg && L1 + L2 <= rem;
      bp += two ? L1 + L2 : L1;
    }
  }
  r.entry = bp;
  const uint32_t c0 = sink.count();
  // fast: 2-symbol steps while bp + 12 < bstop and bp + 30 <= bend.  One
  // loop exit: EOS (the FSM's sticky failure state) drops the bound.
#if HD_BITBUF
  // bb: valid bits MSB-aligned, nb >= 32 of them at the top of every step;
  // nxt: the next staged word, loaded a refill ahead.  The dependent chain
  // of a step is the table read and a 64-bit shift.
  int32_t F = min((int32_t)bstop - 12, (int32_t)bend - 29);
  if ((int32_t)bp < F) {
    uint32_t wi = bp >> 5;
    uint64_t bb = (((uint64_t)ibe[wi] << 32) | ibe[wi + 1]) << (bp & 31u);
    uint32_t nb = 64u - (bp & 31u);
    wi += 2;
    uint32_t nxt = ibe[wi];
    do {
      DCTR(0);
      const uint32_t w = (uint32_t)(bb >> 32);
      uint32_t e = T.lut[w >> (32 - HD_HUFF_LUT_BITS)];
      if (e == 0u) {
        e = long_entry(T, w, 30u);
        if (e == 0xFFFFFFFFu) {
          F = INT32_MIN;
          e = 0u;
        }
      }
      sink.put2(e, (e >> 24) & 3u);
      const uint32_t used = e >> 27;
      bp += used;
      bb <<= used;
      nb -= used;
      const bool need = nb < 32u;
      bb |= need ? ((uint64_t)nxt << (32u - nb)) : 0ull;
      nb += need ? 32u : 0u;
      wi += need ? 1u : 0u;
      nxt = ibe[wi];
    } while ((int32_t)bp < F);
  }
#else
  int32_t F = min((int32_t)bstop - 13, (int32_t)bend - 30);  // bound for q = bp - 1
  uint32_t q = bp - 1u;
  while ((int32_t)q < F) {
    DCTR(0);
    const uint32_t w = win_q(ibe, q);
    uint32_t e = T.lut[w >> (32 - HD_HUFF_LUT_BITS)];
    if (e == 0u) {
      e = long_entry(T, w, 30u);
      if (e == 0xFFFFFFFFu) {
        F = INT32_MIN;
        e = 0u;
      }
    }
    sink.put2(e, (e >> 24) & 3u);
    q += e >> 27;
  }
  bp = q + 1u;
#endif
  bool failed = F == INT32_MIN;
  // checked: to the first boundary >= bstop, or the string's tail
  while (!failed && bp < bstop) {
    const uint32_t rem = bend - bp;
    if (rem == 0) break;
    DCTR(1);
    const uint32_t w = win_at(ibe, bp);
    uint32_t e = T.lut[w >> (32 - HD_HUFF_LUT_BITS)];
    if (e == 0u) {
      e = long_entry(T, w, rem);
      if (e == 0xFFFFFFFFu) {
        failed = true;
        break;
      }
    }
    const uint32_t L1 = (e >> 8) & 31u;
    const uint32_t L2 = (e >> 13) & 7u;
    if (L1 > rem) {  // the tail is a proper prefix of a code
      r.at_end = true;
      r.t = rem;
      r.win = w;
      break;
    }
    const bool two = L2 != 0 && L1 + L2 <= rem && bp + L1 < bstop;
    sink.put2(e, two ? 2u : 1u);
    bp += two ? L1 + L2 : L1;
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

// Tile string holding item q: the last i with sbase[i] <= q.
__device__ __forceinline__ uint32_t find_string(const uint32_t *sbase, uint32_t nstr, uint32_t q) {
  uint32_t lo = 0, hi = nstr - 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (sbase[mid] <= q) lo = mid; else hi = mid - 1;
  }
  return lo;
}

struct DecShared {
  uint32_t ibe[IBUF_BYTES / 4 + 4];  // 16 spare bytes, then the round's input (big-endian words)
  DecTables T;
  uint32_t sa[DEC_NS + 1];       // tile string offsets
  uint32_t sbase[DEC_NS + 1];    // first item of each tile string
  uint32_t es[DEC_NT], xs[DEC_NT], cs[DEC_NT];  // per item of the round: entry, exit, symbols
  uint32_t seg[DEC_NT];          // symbols of the item's string through the item
  uint32_t hist[128];
  uint16_t perm[DEC_NT];
  uint8_t head[DEC_NT];          // item is its string's first (k = 0)
  uint8_t unsettled[DEC_NT];
  uint32_t red[2 * (DEC_NT / 64)];
  uint32_t qmax;                 // round: end of the output image (relative)
  uint32_t rinfo[2];             // round: first input byte (incl. warm-up), string of the first item
  uint32_t carry[2];             // {exit, symbols so far} of the string running into the next round
};

// One persistent workgroup per group of tiles.  AUTO: engine slots (written
// to dst_off), staged in LDS per round when the round's slot range fits;
// else caller slots written directly, capacity-checked.
template <bool AUTO>
__global__ __launch_bounds__(DEC_NT) void k_decode(const uint8_t *__restrict__ src,
                                                   const uint32_t *__restrict__ off, uint32_t n,
                                                   uint8_t *__restrict__ dst, uint64_t dst_cap,
                                                   uint32_t *__restrict__ dst_off,
                                                   int32_t *__restrict__ status,
                                                   uint16_t *__restrict__ fstate_out,
                                                   uint8_t *__restrict__ flags_out) {
  __shared__ DecShared S;
  __shared__ uint32_t obuf[(AUTO && HD_DEC_OUTSTAGE) ? DEC_OBUF / 4 + 64 : 1];
  const uint32_t tid = threadIdx.x;
  const lds_u32 *ibe = (const lds_u32 *)S.ibe;
  lds_u8 *junk = (lds_u8 *)(obuf + ((AUTO && HD_DEC_OUTSTAGE) ? DEC_OBUF / 4 : 0)) + 4u * (tid & 63u);
  stage_dec_tables(S.T, DEC_NT);
  const uint32_t off0 = off[0];
  unsigned long long ts = HD_DIAG_STAMPS ? __builtin_amdgcn_s_memtime() : 0ull;
  (void)ts;
  for (uint32_t t0 = blockIdx.x * DEC_NS; t0 < n; t0 += gridDim.x * DEC_NS) {
    COUNT(11, 1);
    const uint32_t nstr = min(n - t0, (uint32_t)DEC_NS);
    // ---- tile strings -> offsets, engine slots, items per string
    uint32_t m2[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t i = 2u * tid + h;
      m2[h] = 0;
      if (i < nstr) {
        const uint32_t a = off[t0 + i], b = off[t0 + i + 1];
        S.sa[i] = a;
        if (AUTO) dst_off[t0 + i] = (uint32_t)auto_slot(a - off0, t0 + i);
        m2[h] = b - a > PIECE_BYTES ? (b - a + PIECE_BYTES - 1u) / PIECE_BYTES : 1u;
        if (i == nstr - 1) {
          S.sa[nstr] = b;
          if (AUTO && t0 + nstr == n) dst_off[n] = (uint32_t)auto_slot(b - off0, n);
        }
      }
    }
    {
      uint32_t tot;
      const uint32_t ex = block_excl_scan<DEC_NT>(m2[0] + m2[1], S.red, &tot);
      S.sbase[2u * tid] = ex;
      S.sbase[2u * tid + 1] = ex + m2[0];
      if (tid == 0) {
        S.sbase[DEC_NS] = tot;
        S.carry[0] = 0;
        S.carry[1] = 0;
      }
      __syncthreads();
    }
    const uint32_t nitems = S.sbase[DEC_NS];
    uint32_t IB_prev = 0;
    STAMP(0, ts);
    for (uint32_t r0 = 0; r0 < nitems; r0 += DEC_NT) {
      COUNT(10, 1);
      const uint32_t nr = min(nitems - r0, (uint32_t)DEC_NT);  // items this round
      // ---- items of the round in order (thread t <-> item r0 + t): sort key,
      // head flags, the round's first input byte
      uint32_t key = 0;
      if (tid < nr) {
        const uint32_t q = r0 + tid;
        const uint32_t i = find_string(S.sbase, nstr, q);
        const uint32_t k = q - S.sbase[i];
        const uint32_t a = S.sa[i], b = S.sa[i + 1];
        const uint32_t s = a + PIECE_BYTES * k;
        key = min(b - s, PIECE_BYTES) + (k ? SUB_OV : 0u);
        S.head[tid] = k == 0;
        if (tid == 0) {
          S.rinfo[0] = k ? s - SUB_OV : s;
          S.rinfo[1] = i;
        }
      }
      if (tid < 128) S.hist[tid] = 0;
      if (tid == 0) S.qmax = 0;
      __syncthreads();
      const uint32_t A = S.rinfo[0], i0 = S.rinfo[1];
      const uint32_t IB = A & ~15u;
      const uint32_t IBX = IB - 16u;  // bit positions: 8 * (byte - IBX) >= 128
      {  // ---- stage the round's input [IB, IB + IBUF_BYTES) within the pool contract
        const uint32_t lim = ((S.sa[nstr] + 15u) & ~15u) + 16u;
        const uint32_t nchunk = (min(IB + IBUF_BYTES, lim) - IB) >> 4;
        const uint4 *g = reinterpret_cast<const uint4 *>(src + IB);
        for (uint32_t c = tid; c < nchunk; c += DEC_NT) {
          const uint4 v = g[c];
          reinterpret_cast<uint4 *>(S.ibe)[c + 1] =
              make_uint4(__builtin_bswap32(v.x), __builtin_bswap32(v.y), __builtin_bswap32(v.z),
                         __builtin_bswap32(v.w));
        }
      }
      // the carried exit is a bit position of the previous round's staging
      uint32_t carry_exit = S.carry[0];
      if (carry_exit < NOSPEC) carry_exit -= 8u * (IB - IB_prev);
      IB_prev = IB;
      const uint32_t carry_cnt = S.carry[1];
      // ---- the round's output image [P, U) (uniform)
      uint64_t OB = 0, P = 0;
      bool staged = false;
      if (AUTO) {
        P = auto_slot(S.sa[i0] - off0, t0 + i0) + (S.head[0] ? 0u : carry_cnt);
        const uint32_t il = find_string(S.sbase, nstr, r0 + nr - 1);
        const uint64_t U = auto_slot(S.sa[il + 1] - off0, t0 + il + 1);
        OB = P & ~(uint64_t)15u;
        staged = HD_DEC_OUTSTAGE && U - OB <= DEC_OBUF && U <= dst_cap;
      }
      // ---- length-sorted assignment: thread t decodes item r0 + perm[t]
      uint32_t rank = 0;
      if (tid < nr) rank = atomicAdd(&S.hist[key], 1u);
      __syncthreads();
      {
        uint32_t tot;
        const uint32_t h = tid < 128 ? S.hist[tid] : 0u;
        const uint32_t ex = block_excl_scan<DEC_NT>(h, S.red, &tot);
        if (tid < 128) S.hist[tid] = ex;
        __syncthreads();
        if (tid < nr) S.perm[S.hist[key] + rank] = (uint16_t)tid;
        __syncthreads();
      }
      STAMP(1, ts);
      const bool valid = tid < nr;
      const uint32_t u = valid ? S.perm[tid] : 0u;
      const uint32_t q = r0 + u;
      const uint32_t i = find_string(S.sbase, nstr, q), j = t0 + i;
      const uint32_t k = q - S.sbase[i];
      const uint32_t a = S.sa[i], b = S.sa[i + 1];
      const uint32_t s = a + PIECE_BYTES * k;
      const bool last = s + PIECE_BYTES >= b;
      const uint32_t bseg = 8u * (s - IBX);
      const uint32_t bend = 8u * (min(b, s + PIECE_BYTES + 32u) - IBX);
      const uint32_t bstop = last ? bend : 8u * (s + PIECE_BYTES - IBX);
      bool slot_ovf = false;  // AUTO: the string's slot is beyond dst_cap
      uint64_t o = 0;
      uint32_t cap = 0;
      if (AUTO) {
        o = auto_slot(a - off0, j);
        slot_ovf = auto_slot(b - off0, j + 1) > dst_cap;
      } else {
        o = dst_off[j];
        cap = dst_off[j + 1] - (uint32_t)o;
      }
      uint32_t qend = 0;  // end of this lane's output (relative to OB)
      uint32_t dctr[3] = {0, 0, 0};
      // ---- pass 1: k = 0 exact (written); k > 0 speculative count
      if (valid) {
        SubOut r;
        bool ovf = false;
        if (k == 0) {
          if (slot_ovf) {
            r.entry = r.exit = XFAIL;
            r.cnt = 0;
            ovf = true;
          } else if (!AUTO) {
            CheckedSink sk;
            sk.init(dst + o, cap);
            r = decode_item<false>(S.T, ibe, bseg, bseg, bstop, bend, sk, dctr);
            ovf = sk.ovf;
          } else if (staged) {
            LdsSink<false> sk;
            sk.p = (lds_u8 *)obuf + (uint32_t)(o - OB);
            r = decode_item<false>(S.T, ibe, bseg, bseg, bstop, bend, sk, dctr);
            qend = (uint32_t)(o - OB) + r.cnt;
          } else {
            DwordSink sk;
            sk.init(dst + o);
            r = decode_item<false>(S.T, ibe, bseg, bseg, bstop, bend, sk, dctr);
            sk.finish(last);
          }
          if (last) {
            uint32_t fs = 0, fl = 0;
            status[j] = finish_string(S.T, r, r.cnt, ovf, &fs, &fl);
            if (fstate_out) fstate_out[j] = (uint16_t)fs;
            if (flags_out) flags_out[j] = (uint8_t)fl;
          }
        } else {
          NullSink nk;
          r = decode_item<true>(S.T, ibe, bseg - 8u * SUB_OV, bseg, bstop, bend, nk, dctr);
        }
        S.es[u] = r.entry;
        S.xs[u] = r.exit;
        S.cs[u] = r.cnt;
      }
#if HD_DIAG_STAMPS
      {
        uint32_t m0 = dctr[0], m1 = dctr[1], m2x = dctr[2];
        for (int d = 32; d; d >>= 1) {
          m0 = max(m0, (uint32_t)__shfl_xor(m0, d, 64));
          m1 = max(m1, (uint32_t)__shfl_xor(m1, d, 64));
          m2x = max(m2x, (uint32_t)__shfl_xor(m2x, d, 64));
        }
        if ((tid & 63) == 0) {
          atomicAdd(&g_stamps[blockIdx.x & 4095][12], (unsigned long long)m0);
          atomicAdd(&g_stamps[blockIdx.x & 4095][13], (unsigned long long)m1);
          atomicAdd(&g_stamps[blockIdx.x & 4095][14], (unsigned long long)m2x);
        }
      }
#endif
      __syncthreads();
      STAMP(2, ts);
      // ---- verify / redo: entry of item (i, k > 0) must equal the exit of
      // item (i, k - 1), the previous item (or the carry).  A mismatched
      // item is re-decoded once its predecessor is settled (not itself
      // mismatched in this iteration); the first item of the round and k = 0
      // items are always settled, so each iteration settles at least the
      // first mismatch.
      for (uint32_t it = 0; it <= DEC_NT; ++it) {
        bool mism = false;
        uint32_t pred = 0;
        if (valid && k > 0) {
          pred = u ? S.xs[u - 1] : carry_exit;
          const uint32_t e0 = S.es[u];
          mism = e0 != pred || e0 == XUNKNOWN;
        }
        if (valid) S.unsettled[u] = mism ? 1u : 0u;
        const bool any = __syncthreads_or(mism);
#if HD_DIAG_STAMPS
        { const unsigned long long nm = __syncthreads_count(mism); COUNT(9, nm); COUNT(8, 1); }
#endif
        if (!any) break;
        if (mism && (u == 0 || !S.unsettled[u - 1])) {
          SubOut rr;
          rr.cnt = 0;
          if (pred == XFAIL || pred == XUNKNOWN) {
            rr.entry = rr.exit = XFAIL;
          } else {
            NullSink nk;
            rr = decode_item<false>(S.T, ibe, pred, bseg, bstop, bend, nk, dctr);
          }
          S.es[u] = rr.entry;
          S.xs[u] = rr.exit;
          S.cs[u] = rr.cnt;
        }
        __syncthreads();
      }
      STAMP(3, ts);
      // ---- symbols of each string through each item: segmented inclusive
      // scan in item order, segments headed by k = 0 items; the first
      // segment continues the carry.
      {
        const bool live = tid < nr;
        const uint32_t v = live ? S.cs[tid] : 0u;
        const int32_t h = (!live || S.head[tid]) ? (int32_t)tid : -1;
        uint32_t ps = v;
        int32_t hm = h;
        const uint32_t lane = tid & 63u, wv = tid >> 6;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
          const uint32_t o2 = __shfl_up(ps, d, 64);
          const int32_t oh = __shfl_up(hm, d, 64);
          if (lane >= d) {
            ps += o2;
            hm = max(hm, oh);
          }
        }
        if (lane == 63) {
          S.red[wv] = ps;
          S.red[DEC_NT / 64 + wv] = (uint32_t)hm;
        }
        __syncthreads();
        for (uint32_t w = 0; w < wv; ++w) {
          ps += S.red[w];
          hm = max(hm, (int32_t)S.red[DEC_NT / 64 + w]);
        }
        S.seg[tid] = ps;  // inclusive prefix
        __syncthreads();
        const uint32_t base = hm >= 0 ? S.seg[hm] - (hm < (int32_t)nr ? S.cs[hm] : 0u) : 0u - carry_cnt;
        __syncthreads();
        S.seg[tid] = ps - base;
        __syncthreads();
      }
      STAMP(4, ts);
      // ---- pass 2: k > 0 exact, at the string's running symbol count
      if (valid && k > 0) {
        const uint32_t soff = S.seg[u] - S.cs[u];
        const uint32_t e0 = S.es[u];
        SubOut r;
        r.entry = r.exit = XFAIL;
        r.cnt = 0;
        r.t = r.win = 0;
        r.at_end = false;
        bool ovf = AUTO && slot_ovf;
        if (e0 != XFAIL && !ovf) {
          if (!AUTO) {
            CheckedSink sk;
            sk.init(dst + o + min(soff, cap), cap > soff ? cap - soff : 0u);
            r = decode_item<false>(S.T, ibe, e0, bseg, bstop, bend, sk, dctr);
            ovf = soff + r.cnt > cap;  // this piece or an earlier one overflowed
          } else if (staged) {
            LdsSink<true> sk;
            sk.p = (lds_u8 *)obuf + (uint32_t)(o + soff - OB);
            sk.junk = junk;
            r = decode_item<false>(S.T, ibe, e0, bseg, bstop, bend, sk, dctr);
            qend = (uint32_t)(o + soff - OB) + r.cnt;
          } else {
            GlobalSink sk;
            sk.p = dst + o + soff;
            r = decode_item<false>(S.T, ibe, e0, bseg, bstop, bend, sk, dctr);
          }
        } else if (!AUTO) {
          ovf = soff > cap;
        }
        if (last) {
          uint32_t fs = 0, fl = 0;
          status[j] = finish_string(S.T, r, soff + r.cnt, ovf, &fs, &fl);
          if (fstate_out) fstate_out[j] = (uint16_t)fs;
          if (flags_out) flags_out[j] = (uint8_t)fl;
        }
      }
      if (staged && qend) atomicMax(&S.qmax, qend);
      __syncthreads();
      STAMP(5, ts);
      // ---- carry the string running into the next round
      if (tid == 0) {
        S.carry[0] = S.xs[nr - 1];
        S.carry[1] = S.seg[nr - 1];
      }
      // ---- store the round's image [P, OB + qmax): whole 16-byte words,
      // partial words at either end bytewise (their other bytes belong to
      // the neighbouring rounds)
      if (staged) {
        const uint64_t hi = OB + S.qmax;
        const lds_u8 *ob = (const lds_u8 *)obuf;
        if (hi > P) {
          const uint64_t wlo = (P + 15u) & ~(uint64_t)15u, whi = hi & ~(uint64_t)15u;
          if (wlo <= whi) {
            const uint32_t nwords = (uint32_t)((whi - wlo) >> 4);
            uint4 *g = reinterpret_cast<uint4 *>(dst + wlo);
            const uint4 *l = reinterpret_cast<const uint4 *>(obuf) + ((wlo - OB) >> 4);
            for (uint32_t c = tid; c < nwords; c += DEC_NT) g[c] = l[c];
            if (tid < wlo - P) dst[P + tid] = ob[P - OB + tid];
            if (tid >= 16 && tid - 16 < hi - whi) dst[whi + tid - 16] = ob[whi - OB + tid - 16];
          } else if (tid < hi - P) {
            dst[P + tid] = ob[P - OB + tid];
          }
        }
      }
      __syncthreads();
      STAMP(6, ts);
    }
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
template <auto KERNEL, int BS, int UNIT = BS>  // UNIT: items per workgroup task
static uint32_t persistent_grid(uint32_t n) {
  static uint32_t cap = 0;  // one per kernel
  if (cap == 0) cap = resident_blocks(KERNEL, BS);
  const uint32_t g = (n + UNIT - 1) / UNIT;
  return g < cap ? g : cap;
}

static int hip_rv(hipError_t e) {
  if (e == hipSuccess) return 0;
  fprintf(stderr, "nghttp2_amd_hd: HIP error %s\n", hipGetErrorString(e));
  return NGHTTP2_AMD_ERR_FATAL;
}

#if HD_DIAG_STAMPS
extern "C" __attribute__((visibility("default"))) int nghttp2_amd_hd__diag_stamps(void *out, int reset) {
  if (reset) {
    static unsigned long long z[4096][16];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z));
  }
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 4096 * 16);
}
#endif

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
  hipLaunchKernelGGL(k_decode<false>, dim3(persistent_grid<k_decode<false>, DEC_NT, DEC_NS>(n)), dim3(DEC_NT), 0,
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
  hipLaunchKernelGGL(k_decode<true>, dim3(persistent_grid<k_decode<true>, DEC_NT, DEC_NS>(n)), dim3(DEC_NT), 0, st, src, src_off,
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
