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
//   k_decode_items  decode_batch_auto: persistent waves, tasks of 64 strings,
//                   rounds of up to 64 items (a string, or a 32/40/64-byte
//                   piece of a long one, warmed up and verified; budgeted
//                   instances cut a round at an input-byte budget); a 13- or
//                   14-bit two-symbol lookup in LDS and a register bit
//                   buffer; symbols through
//                   a per-lane LDS region, stored back to back per task; the
//                   final {fstate, flags} of the reference's nibble FSM
//                   (lib/nghttp2_hd_huffman.c:122-136) rebuilt exactly from
//                   the undecoded tail bits (DESIGN.md "decode state")
//   k_decode        caller slots (decode_batch), and the round-1 engine-slot
//                   kernel kept for A/B
//   k_decode_fsm    the reference's nibble FSM itself (257x16 table in LDS),
//                   kept as the exact cross-check path and for chunked calls
//   k_slot_len / k_scan_tiles / k_scan_apply   tight decode slots
//                   (floor(8E/5)+1 each)
//   k_frame_len / k_frame_copy   HPACK string literals (emit_string)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <type_traits>

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

// Ablation switch (tools/diag builds variants; the product uses the default)

#ifndef HD_DIAG_STAMPS
#define HD_DIAG_STAMPS 0   // diagnostic build only: per-phase s_memtime sums
#endif
#if HD_DIAG_STAMPS
// Diagnostic build only: per-wave phase cycles of k_decode (s_memtime deltas
// kept in SGPRs, one row per wave written once at exit).  Slots: 0 task
// setup, 1 staging, 2 pass 1, 3 verify, 4 scan, 5 pass 2, 6 round end,
// 7 lifetime, 8 tasks, 9 rounds.
__device__ unsigned long long g_stamps[4096][20];
#define WSTAMP(slot)                                                           \
  do {                                                                         \
    const unsigned long long t1_ = __builtin_amdgcn_s_memtime();               \
    wst[slot] += t1_ - wt0;                                                    \
    wt0 = t1_;                                                                 \
  } while (0)
#define WCOUNT(slot) (++wst[slot])
#define WSTAMP_INIT() unsigned long long wst[13] = {}, wt0 = __builtin_amdgcn_s_memtime(), wbirth = wt0
#define WSTAMP_FLUSH() WSTAMP_FLUSH_W(DEC_WAVES)
#define WSTAMP_FLUSH_W(NW)                                                     \
  do {                                                                         \
    wst[7] = __builtin_amdgcn_s_memtime() - wbirth;                            \
    unsigned long long c_[4];                                                  \
    for (int k_ = 0; k_ < 4; ++k_) {                                           \
      unsigned long long t_ = 0;                                               \
      for (int l_ = 0; l_ < 64; ++l_) t_ += __builtin_amdgcn_readlane(dctr[k_], l_); \
      c_[k_] = t_;                                                             \
    }                                                                          \
    if (lane == 0) {                                                           \
      for (int s_ = 0; s_ < 13; ++s_) g_stamps[(blockIdx.x * (NW) + wv) & 4095][s_] = wst[s_]; \
      for (int k_ = 0; k_ < 4; ++k_) g_stamps[(blockIdx.x * (NW) + wv) & 4095][13 + k_] = c_[k_]; \
    }                                                                          \
  } while (0)
// counts wave iterations: only the first active lane counts (the flush sums lanes)
#define DCTR(k)                                                                \
  do {                                                                         \
    const uint32_t l_ = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); \
    if (__builtin_amdgcn_readfirstlane(l_) == l_) ++dctr[k];                   \
  } while (0)
#define DD_SARGS , unsigned long long *wst, unsigned long long &wt0
#define DD_SPASS , wst, wt0
#else
#define DD_SARGS
#define DD_SPASS
#define WSTAMP(slot) do { } while (0)
#define WCOUNT(slot) do { } while (0)
#define WSTAMP_INIT() do { } while (0)
#define WSTAMP_FLUSH() do { } while (0)
#define WSTAMP_FLUSH_W(NW) do { } while (0)
#define DCTR(k) do { } while (0)
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
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;

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

// ---------------------------------------------------------------------------
// encode, pass 2: bit packing   (lib/nghttp2_hd_huffman.c:45-104)
// ---------------------------------------------------------------------------
// Bit-pack one string [a, b) MSB-first (lib/nghttp2_hd_huffman.c:57-84) into
// out_base[o ..], padding the last byte with the EOS prefix (:95-101).
// ---------------------------------------------------------------------------
// encode (lib/nghttp2_hd_huffman.c:34-104), balanced by raw bytes.  A wave
// owns 64 consecutive strings (lane i <-> string i) and walks their PIECES
// of ENC_PIECE raw bytes in rounds of 64 (one per lane), so every lane
// handles <= 32 input bytes per round whatever the string lengths.
// ---------------------------------------------------------------------------
#ifndef ENC_PIECE
#define ENC_PIECE 32u
#endif
#define ENC_PW (ENC_PIECE / 4)       // dwords per piece
#define ENC_PC (ENC_PIECE / 16 + 1)  // aligned chunks covering a piece
#define ENC_WAVES 4                  // waves per encode workgroup (tile = 256 strings)
#define ENC_REGION 4096u             // per-wave LDS output staging (bytes)

struct EncPiece {
  uint32_t i, k, s, e;  // wave string, piece, raw bytes [s, e)
  uint32_t a;           // the string's first raw byte
  bool last;            // the string's last piece
};

// Piece q of the wave's strings: string = first i with P_i > q.
__device__ __forceinline__ EncPiece enc_piece(uint32_t q, uint32_t nstr, uint32_t P_l, uint32_t X_l,
                                              uint32_t a_l, uint32_t b_l) {
  uint32_t lo = 0, hi = nstr - 1u;
#pragma unroll
  for (int st = 0; st < 6; ++st) {
    const uint32_t mid = (lo + hi) >> 1;
    const uint32_t pm = __shfl(P_l, mid, 64);
    if (pm > q) hi = mid; else lo = mid + 1u;
  }
  EncPiece p;
  p.i = min(lo, nstr - 1u);
  p.k = q - __shfl(X_l, p.i, 64);
  const uint32_t a = __shfl(a_l, p.i, 64), b = __shfl(b_l, p.i, 64);
  p.a = a;
  p.s = a + ENC_PIECE * p.k;
  p.e = min(b, p.s + ENC_PIECE);
  p.last = p.s + ENC_PIECE >= b;
  return p;
}

// A piece's bytes, realigned so that byte j of the piece is byte j of w[]:
// the three aligned 16-byte chunks covering it are loaded (only those that
// hold piece bytes -- the pool contract ends at align16(off[n]) + 16), then
// shifted by the piece's offset in its first chunk.
struct PieceBytes {
  uint32_t w[ENC_PW];
  uint32_t len;  // piece bytes (<= ENC_PIECE)
  __device__ __forceinline__ void load(const uint8_t *src, const EncPiece &p, bool valid) {
    const uint32_t c0 = p.s & ~15u;
    const uint4 *g = reinterpret_cast<const uint4 *>(src + c0);
    len = valid ? p.e - p.s : 0u;
    uint32_t x[4 * ENC_PC];
#pragma unroll
    for (int c = 0; c < ENC_PC; ++c) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (valid && p.e > c0 + 16u * c) v = g[c];
      x[4 * c] = v.x; x[4 * c + 1] = v.y; x[4 * c + 2] = v.z; x[4 * c + 3] = v.w;
    }
    const uint32_t d = p.s & 15u, q = d >> 2, r = 8u * (d & 3u);
    // y[k] = x[k + q] for k = 0..ENC_PW (q in 0..3): selects, no runtime indexing
    uint32_t y[ENC_PW + 1];
#pragma unroll
    for (int k = 0; k <= ENC_PW; ++k) {
      const uint32_t a0 = x[k], a1 = x[k + 1], a2 = x[k + 2], a3 = (k + 3 < 4 * ENC_PC) ? x[k + 3] : 0u;
      y[k] = (q & 2u) ? ((q & 1u) ? a3 : a2) : ((q & 1u) ? a1 : a0);
    }
#pragma unroll
    for (int k = 0; k < ENC_PW; ++k)
      w[k] = r ? (uint32_t)((((uint64_t)y[k + 1] << 32) | y[k]) >> r) : y[k];
  }
  __device__ __forceinline__ uint32_t byte(int j) const { return (w[j >> 2] >> (8 * (j & 3))) & 0xFFu; }
};

// Code bits of a piece; jmax: the wave's longest piece (uniform loop bound).
__device__ __forceinline__ uint32_t piece_bits(const PieceBytes &pb, const uint8_t *lenT, uint32_t jmax) {
  uint32_t bits = 0;
#pragma unroll
  for (int k = 0; k < ENC_PW; ++k) {
    if ((uint32_t)(4 * k) < jmax) {  // uniform
      const uint32_t wd = pb.w[k];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t L = lenT[(wd >> (8 * b)) & 0xFFu];
        bits += ((uint32_t)(4 * k + b) < pb.len) ? L : 0u;
      }
    }
  }
  return bits;
}

// Uniform maximum / minimum over the wave.
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int d = 32; d; d >>= 1) v = max(v, (uint32_t)__shfl_xor(v, d, 64));
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
  for (int d = 32; d; d >>= 1) v = min(v, (uint32_t)__shfl_xor(v, d, 64));
  return __builtin_amdgcn_readfirstlane(v);
}

// Per-string encoded lengths (and per-tile sums): pass 1 of the batch.
// Piece slot in the optional per-piece bit-count array: the pieces before
// string s number <= (off[s] - off[0]) / ENC_PIECE + s, so
// slot(s, k) = (off[s] - off[0]) / ENC_PIECE + s + k is unique and
// increasing; the array holds enc_piece_slots(raw_bytes, n) entries.
__device__ __host__ __forceinline__ uint64_t enc_piece_slot(uint32_t rel, uint32_t s, uint32_t k) {
  return (uint64_t)(rel / ENC_PIECE) + s + k;
}

__global__ __launch_bounds__(WG) void k_enc_count_r1(const uint8_t *__restrict__ src,
                                                  const uint32_t *__restrict__ off,
                                                  uint32_t n,
                                                  uint32_t *__restrict__ out_len,
                                                  uint32_t *__restrict__ tile_sums,
                                                  uint16_t *__restrict__ piece_bits_out,
                                                  int bits_out) {
  __shared__ uint8_t lenT[256];
  __shared__ uint32_t sbits[ENC_WAVES][64];
  __shared__ uint32_t red[WG / 64];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  lenT[threadIdx.x] = dev::hd_huff_enc_len[threadIdx.x];
  sbits[wv][lane] = 0;
  __syncthreads();
  const uint32_t t0 = blockIdx.x * WG + 64u * wv;  // the wave's strings
  uint32_t e = 0;
  if (t0 < n) {
    const uint32_t nstr = min(n - t0, 64u);
    const bool sl = lane < nstr;
    const uint32_t a_l = sl ? off[t0 + lane] : 0u, b_l = sl ? off[t0 + lane + 1] : 0u;
    const uint32_t m_l = sl ? max(1u, (b_l - a_l + ENC_PIECE - 1u) / ENC_PIECE) : 0u;
    const uint32_t P_l = wave_incl_scan(m_l), X_l = P_l - m_l;
    const uint32_t M = __builtin_amdgcn_readlane(P_l, 63);
    const uint32_t off0 = off[0];
    for (uint32_t r0 = 0; r0 < M; r0 += 64u) {
      const bool valid = r0 + lane < M;
      const EncPiece p = enc_piece(r0 + lane, nstr, P_l, X_l, a_l, b_l);
      PieceBytes pb;
      pb.load(src, p, valid);
      const uint32_t bits = piece_bits(pb, lenT, wave_max(pb.len));
      if (valid) {
        atomicAdd(&sbits[wv][p.i], bits);
        if (piece_bits_out)
          piece_bits_out[enc_piece_slot(p.a - off0, t0 + p.i, p.k)] = (uint16_t)bits;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (sl) {
      e = (sbits[wv][lane] + 7u) >> 3;
      if (out_len) out_len[t0 + lane] = bits_out ? sbits[wv][lane] : e;
    }
  }
  if (tile_sums) {
    uint32_t tot;
    block_excl_scan<WG>(e, red, &tot);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
  }
}

// Pack (lib/nghttp2_hd_huffman.c:45-104), stream-parallel.  On entry
// dst_off[s] holds string s's code bits (k_enc_count with bits_out); the
// tile prologue turns them into byte offsets (E = ceil(bits / 8)).  A wave
// owns 64 consecutive strings and walks their raw bytes as aligned 16-byte
// chunks, 64 per round (one per lane), whatever the string lengths.
//
// Positions: with P(p) = code bits of the wave's bytes before byte p (a plain
// prefix, no padding), byte p of string s starts at output bit
// 8 * O_s + P(p) - P(a_s).  So a chunk's start = anchor[s] + P(chunk), with
// anchor[s] = 8 * O_s - P(a_s) from one scan over the wave's strings and P
// from one scan over the round's chunk sums.  Inside a chunk a string start
// rounds the position up to a byte; the EOS-prefix padding itself
// (:95-101) is OR'ed in afterwards by the string's own lane, which knows its
// pad = 8 * E - bits.  Codes are appended MSB-first into a 64-bit register
// and completed words OR'ed into the round's LDS image, which goes out as
// whole dwords (zeroed behind the store); the partial word at a round's end
// is carried into the next round, and the dwords at the wave's two ends go
// bytewise.
// ---------------------------------------------------------------------------
#define ENC_RW 1024u  // LDS words per wave image: 1 KB of input at <= 30 bits a byte + edges

__global__ __launch_bounds__(WG) void k_encode_r1(const uint8_t *__restrict__ src,
                                               const uint32_t *__restrict__ off, uint32_t n,
                                               uint8_t *__restrict__ dst, uint64_t dst_cap,
                                               uint32_t *__restrict__ dst_off,
                                               const uint32_t *__restrict__ tile_sums) {
  __shared__ uint2 codeT[512];                   // [256..511] = {0, 0}: bytes outside the wave
  __shared__ uint32_t image[ENC_WAVES][ENC_RW];
  __shared__ uint32_t heads[ENC_WAVES][36];
  __shared__ uint32_t cand[ENC_WAVES][65];
  __shared__ uint32_t o_sh[WG + 1];
  __shared__ uint32_t red[2 * (WG / 64)];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  codeT[threadIdx.x] = make_uint2(dev::hd_huff_enc_code[threadIdx.x], dev::hd_huff_enc_len[threadIdx.x]);
  codeT[256 + threadIdx.x] = make_uint2(0u, 0u);
  lds_u32 *img = (lds_u32 *)image[wv];
  for (uint32_t i = lane; i < ENC_RW; i += 64u) img[i] = 0u;
  const uint32_t s_me = blockIdx.x * WG + threadIdx.x;
  const uint32_t bits_me = s_me < n ? dst_off[s_me] : 0u;
  const uint32_t E_me = (bits_me + 7u) >> 3;
  // the wave's strings (lane = string) and its first chunk, before the tile scan
  const uint32_t t0 = blockIdx.x * WG + 64u * wv;
  const uint32_t nstr = t0 < n ? min(n - t0, 64u) : 0u;
  const bool sl = lane < nstr;
  const uint32_t a_l = sl ? off[t0 + lane] : 0u, b_l = sl ? off[t0 + lane + 1] : 0u;
  const uint32_t A = __builtin_amdgcn_readfirstlane(a_l);
  const uint32_t Z = nstr ? __builtin_amdgcn_readlane(b_l, nstr - 1u) : 0u;
  const uint32_t c_end = (Z + 15u) >> 4;
  uint4 wn = make_uint4(0, 0, 0, 0);  // the next round's chunk (prefetched)
  if ((A >> 4) + lane < c_end) wn = *reinterpret_cast<const uint4 *>(src + (((A >> 4) + lane) << 4));
  // the tile's offset: the tile totals before it (k_enc_count; 16 KB for 1M
  // strings, L2-resident), summed with independent loads in flight, in 64
  // bits (a batch's encoded total may pass the uint32 offset range)
  uint64_t pre = 0;
  {
    uint64_t p8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t t = threadIdx.x;
    for (; t + 7u * WG < blockIdx.x; t += 8u * WG) {
#pragma unroll
      for (int k = 0; k < 8; ++k) p8[k] += tile_sums[t + k * WG];
    }
    for (; t < blockIdx.x; t += WG) pre += tile_sums[t];
#pragma unroll
    for (int k = 0; k < 8; ++k) pre += p8[k];
  }
  uint32_t tot, ptot_lo, ptot_hi;
  // the 64-bit prefix as two 32-bit sums: 256 parts of 23 bits fit 31 bits
  const uint32_t loc = block_excl_scan_sum<WG>(E_me, (uint32_t)(pre & 0x7FFFFFu), red, &tot,
                                               &ptot_lo);  // (barriers)
  {
    uint32_t dummy;
    block_excl_scan_sum<WG>(0u, (uint32_t)(pre >> 23), red, &dummy, &ptot_hi);
  }
  const uint64_t ptot = ((uint64_t)ptot_hi << 23) + ptot_lo;
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
  const uint32_t OA = o_sh[64u * wv], OZ = o_sh[64u * wv + nstr];  // the wave's output bytes
  const uint64_t G0 = 8ull * OA;
  // anchor[s] = 8 (O_s - OA) - P(a_s)   (positions relative to G0)
  const uint32_t P_a = wave_incl_scan(sl ? bits_me : 0u) - (sl ? bits_me : 0u);
  const uint32_t anchor_l = 8u * (o_me - OA) - P_a;
  const uint32_t pad_l = sl ? 8u * E_me - bits_me : 0u;  // EOS-prefix bits after string l
  const uint32_t olast_l = o_me + E_me - 1u;             // its last output byte (if E > 0)
  lds_u32 *hb = (lds_u32 *)heads[wv];
  lds_u32 *cd = (lds_u32 *)cand[wv];
  uint32_t Pc = 0;     // P at the round's first byte
  uint32_t scarry = 0; // 1 + the string running into the round
  uint32_t x = 0;      // output bit at the round's start (relative to G0)
  for (uint32_t cb = A >> 4; cb < c_end; cb += 64u) {
    const bool last_round = cb + 64u >= c_end;
    const uint32_t base = cb << 4;
    const uint64_t WB = (G0 + x) >> 5;  // global word of img[0]
    // ---- string starts in this round (alignment points)
    if (lane < 33u) hb[lane] = 0u;
    cd[lane] = 0u;
    if (lane == 0) cd[64] = 0u;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // a string starting in this round: its head bit, and it holds the first
    // valid byte of every chunk from kf on (chunk 0 of the first round starts
    // at A itself)
    if (sl && a_l < b_l && a_l >= base && a_l - base < 1024u) {
      atomicOr((uint32_t *)&hb[(a_l - base) >> 5], 1u << ((a_l - base) & 31u));
      const uint32_t kf = a_l <= max(base, A) ? 0u : (a_l - base + 15u) >> 4;
      atomicMax((uint32_t *)&cd[kf], lane + 1u);
    }
    const uint32_t p0 = base + 16u * lane;  // my chunk's first byte
    const uint32_t lo = A > p0 ? min(A - p0, 16u) : 0u;
    const uint32_t hi = Z > p0 ? min(Z - p0, 16u) : 0u;
    const uint32_t vm = hi > lo ? ((1u << hi) - 1u) & ~((1u << lo) - 1u) : 0u;
    const uint32_t iv = ~vm << 11;  // bit 11 + j: byte j is outside the wave -> zero entry
    const uint32_t wd[4] = {wn.x, wn.y, wn.z, wn.w};
    if (cb + 64u + lane < c_end) wn = *reinterpret_cast<const uint4 *>(src + p0 + 1024u);
    uint2 cc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t b8 = (j & 3) ? (wd[j >> 2] >> (8 * (j & 3) - 3)) & 0x7F8u : (wd[j >> 2] << 3) & 0x7F8u;
      cc[j] = *(const uint2 *)((const char *)codeT + (b8 | ((iv >> j) & 0x800u)));
    }
    uint32_t S = 0, Lmax = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      S += cc[j].y;
      Lmax = max(Lmax, cc[j].y);
    }
    // ---- my chunk's start: anchor of the string holding its first valid
    // byte (an inclusive max-scan of the start marks), plus P there
    const uint32_t Sinc = wave_incl_scan(S);
    const uint32_t Pme = Pc + Sinc - S;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint32_t sm = wave_incl_max(max(cd[lane], scarry));
    const uint32_t start = __shfl(anchor_l, sm - 1u, 64) + Pme;
    const uint32_t hm = (hb[lane >> 1] >> (16u * (lane & 1u))) & vm & 0xFFFFu;
    const uint32_t hmw = wave_or(hm);  // heads at each byte position, over the wave
    const bool short_codes = __ballot(Lmax > 16u) == 0;
    // ---- emit
    uint32_t endp = start;
    if (vm) {
      const uint64_t gp = G0 + start;
      uint32_t wa = (uint32_t)((gp >> 5) - WB);  // image word
      uint32_t nacc = (uint32_t)gp & 31u;
      uint64_t acc = 0;
#define ENC_ALIGN(J)                                                     \
      if (hmw & (1u << (J))) {  /* some lane starts a string here */     \
        const uint32_t h7 = ((hm >> (J)) & 1u) ? 7u : 0u;                 \
        nacc = (nacc + h7) & ~h7;  /* next byte boundary */               \
      }
#define ENC_APPEND(J)                                                    \
      acc |= ((uint64_t)cc[J].x << 32) >> nacc;                          \
      nacc += cc[J].y;
#define ENC_FLUSH()                                                      \
      if (nacc >= 32u) {                                                 \
        atomicOr((uint32_t *)&img[wa], (uint32_t)(acc >> 32));           \
        ++wa;                                                            \
        acc <<= 32;                                                      \
        nacc -= 32u;                                                     \
      }
      if (short_codes) {
        // every code <= 16 bits: nacc <= 32 on entry to a pair, <= 64 after
#pragma unroll
        for (int j = 0; j < 16; j += 2) {
          ENC_ALIGN(j);
          ENC_APPEND(j);
          ENC_ALIGN(j + 1);
          ENC_APPEND(j + 1);
          ENC_FLUSH();
        }
        ENC_FLUSH();
      } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          ENC_ALIGN(j);
          ENC_APPEND(j);
          ENC_FLUSH();
        }
      }
#undef ENC_ALIGN
#undef ENC_APPEND
#undef ENC_FLUSH
      if (nacc) atomicOr((uint32_t *)&img[wa], (uint32_t)(acc >> 32));
      endp = (uint32_t)(32ull * (WB + wa) + nacc - G0);
    }
    // end of the round: the last lane with input
    const uint64_t live = __ballot(vm != 0);
    uint32_t xe = live ? __builtin_amdgcn_readlane(endp, 63u - __builtin_clzll(live)) : x;
    if (last_round) xe = 8u * (OZ - OA);
    const uint32_t nw = (uint32_t)(((G0 + xe + 31u) >> 5) - WB);
    // ---- EOS-prefix padding of the strings that end in this round
    if (sl && pad_l && b_l - 1u >= base && b_l - 1u - base < 1024u && b_l > a_l) {
      const uint32_t r = (uint32_t)((olast_l >> 2) - WB);
      atomicOr((uint32_t *)&img[r], ((1u << pad_l) - 1u) << (24u - 8u * (olast_l & 3u)));
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // ---- store whole words and zero them; carry a partial last word
    const uint32_t nst = last_round ? nw : (uint32_t)(((G0 + xe) >> 5) - WB);
    for (uint32_t i = lane; i < nst; i += 64u) {
      const uint32_t v = __builtin_bswap32(img[i]);
      img[i] = 0u;
      const uint64_t ga = 4ull * (WB + i);
      if (ga >= OA && ga + 4u <= OZ && ga + 4u <= dst_cap) {
        *reinterpret_cast<uint32_t *>(dst + ga) = v;
      } else {
        for (uint32_t y = 0; y < 4u; ++y) {
          const uint64_t gq = ga + y;
          if (gq >= OA && gq < OZ && gq < dst_cap) dst[gq] = (uint8_t)(v >> (8u * y));
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (!last_round && nst < nw) {  // the partial word moves to img[0]
      const uint32_t cw = img[nst];
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) {
        img[nst] = 0u;
        img[0] = cw;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    Pc += __builtin_amdgcn_readlane(Sinc, 63);
    scarry = max(__builtin_amdgcn_readlane(sm, 63), cd[64]);
    x = xe;
  }
}

// ---------------------------------------------------------------------------
// encode over aligned chunks (the product path): a wave owns 64 consecutive
// strings, i.e. the contiguous raw bytes [A, Z), and walks them as aligned
// 16-byte chunks, 64 per round (one per lane), whatever the string lengths.
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(3))) uint16_t lds_u16;

// Pass 1 (lib/nghttp2_hd_huffman.c:34-43): code bits per string.  With P(x)
// = the code bits of the wave's bytes from its first chunk up to byte x, a
// string's bits are P(b) - P(a): each lane sums its chunk's code lengths
// (in-chunk exclusive prefixes to LDS, 16 bits a byte), a wave scan places
// the chunks, and every string lane reads P at its two ends.  Bytes before
// A or past Z in the edge chunks add the same amount to both ends.
__global__ __launch_bounds__(WG) void k_enc_count(const uint8_t *__restrict__ src,
                                                  const uint32_t *__restrict__ off,
                                                  uint32_t n,
                                                  uint32_t *__restrict__ out_len,
                                                  uint32_t *__restrict__ tile_sums,
                                                  int bits_out) {
  __shared__ uint8_t lenT[256];
  __shared__ alignas(16) uint32_t pre[ENC_WAVES][512];  // a round's prefixes (u16 per byte)
  __shared__ uint32_t red[WG / 64];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  lenT[threadIdx.x] = dev::hd_huff_enc_len[threadIdx.x];
  __syncthreads();
  const uint32_t t0 = blockIdx.x * WG + 64u * wv;  // the wave's strings
  uint32_t e = 0;
  if (t0 < n) {
    const uint32_t nstr = min(n - t0, 64u);
    const bool sl = lane < nstr;
    const uint32_t a_l = sl ? off[t0 + lane] : 0u, b_l = sl ? off[t0 + lane + 1] : 0u;
    const uint32_t A = __builtin_amdgcn_readfirstlane(a_l);
    const uint32_t Z = __builtin_amdgcn_readlane(b_l, nstr - 1u);
    const uint32_t c0 = A >> 4, c_end = (Z + 15u) >> 4;
    lds_u32 *pr = (lds_u32 *)pre[wv];
    const lds_u16 *pr16 = (const lds_u16 *)pre[wv];
    uint32_t Rc = 0, Pa = 0, Pb = 0;
    bool ga = false, gb = false;
    // chunks are loaded two rounds ahead (enough bytes in flight per CU)
    uint4 wn = make_uint4(0, 0, 0, 0), wn2 = make_uint4(0, 0, 0, 0);
    if (c0 + lane < c_end) wn = *reinterpret_cast<const uint4 *>(src + ((c0 + lane) << 4));
    if (c0 + 64u + lane < c_end) wn2 = *reinterpret_cast<const uint4 *>(src + ((c0 + 64u + lane) << 4));
    for (uint32_t cb = c0; cb < c_end; cb += 64u) {
      const uint32_t base = cb << 4;
      const uint32_t wd[4] = {wn.x, wn.y, wn.z, wn.w};
      wn = wn2;
      wn2 = make_uint4(0, 0, 0, 0);
      if (cb + 128u + lane < c_end) wn2 = *reinterpret_cast<const uint4 *>(src + base + 2048u + 16u * lane);
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
      *(lds_u32x4 *)(pr + 8u * lane) = v0;
      *(lds_u32x4 *)(pr + 8u * lane + 4u) = v1;
      const uint32_t Sinc = wave_incl_scan(run), Sx = Sinc - run;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // the string ends in this round: P = chunk start + in-chunk prefix
      const uint32_t ra = a_l - base, rb = b_l - base;
      const uint32_t xa = __shfl(Sx, (ra >> 4) & 63u, 64), xb = __shfl(Sx, (rb >> 4) & 63u, 64);
      if (sl && ra < 1024u) {
        Pa = Rc + xa + pr16[ra];
        ga = true;
      }
      if (sl && rb < 1024u) {
        Pb = Rc + xb + pr16[rb];
        gb = true;
      }
      Rc += __builtin_amdgcn_readlane(Sinc, 63);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    // an end at the last chunk's end (Z on a chunk boundary)
    if (!ga) Pa = Rc;
    if (!gb) Pb = Rc;
    const uint32_t bits = sl ? Pb - Pa : 0u;
    e = (bits + 7u) >> 3;
    if (sl && out_len) out_len[t0 + lane] = bits_out ? bits : e;
  }
  if (tile_sums) {
    uint32_t tot;
    block_excl_scan<WG>(e, red, &tot);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
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
#ifndef EC_SB
#define EC_SB 0  // k_encode: a scheduling barrier after every two dwords of lookups
#endif
#ifndef EC_WPE
#define EC_WPE 4  // k_encode: waves per SIMD the register budget is sized for
#endif
#define EC_M 16u                    // image margin (words): >= 15 bytes x 30 bits
#define EC_RW (EC_M + 1024u + 32u)  // + 1 KB at <= 32 bits a byte + carry + bytes past Z

// OR the MSB-aligned bits {hi, lo} into the image at bit b
__device__ __forceinline__ void ec_or3(lds_u32 *img, uint32_t b, uint32_t hi, uint32_t lo) {
  const uint32_t o = b & 31u;
  lds_u32 *q = img + (b >> 5);
  atomicOr((uint32_t *)&q[0], hi >> o);
  atomicOr((uint32_t *)&q[1], __builtin_amdgcn_alignbit(hi, lo, o));
  atomicOr((uint32_t *)&q[2], __builtin_amdgcn_alignbit(lo, 0u, o));  // (0 when o = 0)
}

__global__ __launch_bounds__(WG, EC_WPE) void k_encode(const uint8_t *__restrict__ src,
                                               const uint32_t *__restrict__ off, uint32_t n,
                                               uint8_t *__restrict__ dst, uint64_t dst_cap,
                                               uint32_t *__restrict__ dst_off,
                                               const uint32_t *__restrict__ tile_sums) {
  __shared__ uint2 codeT[256];  // {code MSB-aligned, length}
  __shared__ uint32_t image[ENC_WAVES][EC_RW];
  __shared__ alignas(16) uint32_t padb[ENC_WAVES][256];  // a round's pad bits (u8 per byte)
  __shared__ uint32_t o_sh[WG + 1];
  __shared__ uint32_t red[2 * (WG / 64)];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  codeT[threadIdx.x] = make_uint2(dev::hd_huff_enc_code[threadIdx.x], dev::hd_huff_enc_len[threadIdx.x]);
  lds_u32 *img = (lds_u32 *)image[wv];
  for (uint32_t i = lane; i < EC_RW; i += 64u) img[i] = 0u;
  lds_u32 *pdw = (lds_u32 *)padb[wv];
  lds_u8 *pdb = (lds_u8 *)padb[wv];
#pragma unroll
  for (uint32_t i = 0; i < 4u; ++i) pdw[lane + 64u * i] = 0u;
  const uint32_t s_me = blockIdx.x * WG + threadIdx.x;
  const uint32_t bits_me = s_me < n ? dst_off[s_me] : 0u;
  const uint32_t E_me = (bits_me + 7u) >> 3;
  const uint32_t t0 = blockIdx.x * WG + 64u * wv;
  const uint32_t nstr = t0 < n ? min(n - t0, 64u) : 0u;
  const bool sl = lane < nstr;
  const uint32_t a_l = sl ? off[t0 + lane] : 0u, b_l = sl ? off[t0 + lane + 1] : 0u;
  const uint32_t A = __builtin_amdgcn_readfirstlane(a_l);
  const uint32_t Z = nstr ? __builtin_amdgcn_readlane(b_l, nstr - 1u) : 0u;
  const uint32_t c0 = A >> 4, c_end = (Z + 15u) >> 4;
  uint4 wn = make_uint4(0, 0, 0, 0);  // the next round's chunk (prefetched)
  if (c0 + lane < c_end) wn = *reinterpret_cast<const uint4 *>(src + ((c0 + lane) << 4));
  // the tile's offset: the tile totals before it (k_enc_count; 16 KB for 1M
  // strings, L2-resident), summed with independent loads in flight, in 64
  // bits (a batch's encoded total may pass the uint32 offset range)
  uint64_t pre = 0;
  {
    uint64_t p8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t t = threadIdx.x;
    for (; t + 7u * WG < blockIdx.x; t += 8u * WG) {
#pragma unroll
      for (int k = 0; k < 8; ++k) p8[k] += tile_sums[t + k * WG];
    }
    for (; t < blockIdx.x; t += WG) pre += tile_sums[t];
#pragma unroll
    for (int k = 0; k < 8; ++k) pre += p8[k];
  }
  uint32_t tot, ptot_lo, ptot_hi;
  // the 64-bit prefix as two 32-bit sums: 256 parts of 23 bits fit 31 bits
  const uint32_t loc = block_excl_scan_sum<WG>(E_me, (uint32_t)(pre & 0x7FFFFFu), red, &tot,
                                               &ptot_lo);  // (barriers)
  {
    uint32_t dummy;
    block_excl_scan_sum<WG>(0u, (uint32_t)(pre >> 23), red, &dummy, &ptot_hi);
  }
  const uint64_t ptot = ((uint64_t)ptot_hi << 23) + ptot_lo;
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
  const uint32_t OA = o_sh[64u * wv], OZ = o_sh[64u * wv + nstr];  // the wave's output bytes
  const uint64_t G0 = 8ull * OA;
  const uint32_t pad_l = sl ? 8u * E_me - bits_me : 0u;  // EOS-prefix bits after string l
  const uint32_t olast_l = o_me + E_me - 1u;             // its last output byte (if E > 0)
  const uint32_t tail_l = b_l - 1u;                      // its last raw byte
  uint32_t x = 0;  // output bit of the round's first wave byte (relative to G0)
  for (uint32_t cb = c0; cb < c_end; cb += 64u) {
    const bool first = cb == c0, last_round = cb + 64u >= c_end;
    const uint32_t base = cb << 4;
    const uint64_t WB = (G0 + x) >> 5;  // global word of img[EC_M]
    // ---- pads of the strings ending in this round, at their last raw byte
    const bool tl = sl && pad_l && b_l > a_l && tail_l - base < 1024u;
    if (tl) pdb[tail_l - base] = (uint8_t)pad_l;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t p0 = base + 16u * lane;
    const bool act = p0 < Z;  // (lanes past the wave's last chunk: nothing)
    const uint32_t wd[4] = {wn.x, wn.y, wn.z, wn.w};
    wn = make_uint4(0, 0, 0, 0);
    if (cb + 64u + lane < c_end) wn = *reinterpret_cast<const uint4 *>(src + p0 + 1024u);
    const u32x4 pdv = *(const lds_u32x4 *)(pdw + 4u * lane);
    const uint32_t pd[4] = {pdv.x, pdv.y, pdv.z, pdv.w};
#define EC_B8(j) (((j) & 3) ? (wd[(j) >> 2] >> (8 * ((j) & 3) - 3)) & 0x7F8u : (wd[(j) >> 2] << 3) & 0x7F8u)
    // per input dword: four codes (+ the pad at a string's last byte) ->
    // two pairs {pc, pl} (MSB-aligned, < 32 bits) -> one quad {qh:qo, ql}
    uint32_t qh[4], qo[4], ql[4], plx = 0;
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
      if (EC_SB && (m & 1)) __builtin_amdgcn_sched_barrier(0);  // (bounds the lookups in flight)
    }
    const uint32_t S = act ? ql[0] + ql[1] + ql[2] + ql[3] : 0u;
    const bool longp = __ballot(act && plx > 31u) != 0;  // a pair of 32 bits or more: bytewise
    // ---- the first chunk's bytes before A go before the wave's first bit
    // (no pads there)
    uint32_t RA = 0;
    if (first) {
      const uint32_t k = A & 15u;
      uint32_t ra = 0;
#pragma unroll
      for (int j = 0; j < 15; ++j)
        if ((uint32_t)j < k) ra += ((const uint2 *)((const char *)codeT + EC_B8(j)))->y;
      RA = __builtin_amdgcn_readfirstlane(ra);
    }
    const uint32_t Sinc = wave_incl_scan(S);
    // my chunk's first bit in the image (img[0] = global word WB - EC_M)
    const uint32_t ib0 = (uint32_t)(G0 + x - 32ull * WB) + 32u * EC_M + (Sinc - S) - RA;
    if (act) {
      if (!longp) {
        uint32_t b = ib0;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          ec_or3(img, b, qh[m], qo[m]);
          b += ql[m];
        }
      } else {  // a code of <= 37 bits, MSB-aligned in 64; one dword at a time
        uint32_t b = ib0;
#pragma unroll 1
        for (uint32_t m = 0; m < 4u; ++m) {
          const uint32_t w = m == 0 ? wd[0] : m == 1 ? wd[1] : m == 2 ? wd[2] : wd[3];
          const uint32_t pw = m == 0 ? pd[0] : m == 1 ? pd[1] : m == 2 ? pd[2] : pd[3];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const uint32_t b8 = u ? (w >> (8 * u - 3)) & 0x7F8u : (w << 3) & 0x7F8u;
            const uint2 cj = *(const uint2 *)((const char *)codeT + b8);
            ec_or3(img, b, cj.x, 0u);
            b += cj.y + ((pw >> (8 * u)) & 0xFFu);
          }
        }
      }
    }
#undef EC_B8
    // ---- EOS-prefix padding (all ones) of the strings that end in this round
    if (tl) {
      const uint32_t r = (uint32_t)((olast_l >> 2) - WB) + EC_M;
      atomicOr((uint32_t *)&img[r], ((1u << pad_l) - 1u) << (24u - 8u * (olast_l & 3u)));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // ---- store whole words and zero them; carry a partial last word
    const uint32_t xe = last_round ? 8u * (OZ - OA) : x + __builtin_amdgcn_readlane(Sinc, 63) - RA;
    const uint32_t nw = (uint32_t)(((G0 + xe + 31u) >> 5) - WB);
    const uint32_t nst = last_round ? nw : (uint32_t)(((G0 + xe) >> 5) - WB);
    // words [ilo, ihi) lie inside the wave's output [OA, OZ) (<= dst_cap by
    // the tile check); the others hold bytes of the neighbouring waves
    const uint32_t ilo = (uint32_t)(((uint64_t)OA + 3u) / 4u - min(WB, ((uint64_t)OA + 3u) / 4u));
    const uint32_t ihi = (uint32_t)((uint64_t)OZ / 4u > WB ? (uint64_t)OZ / 4u - WB : 0u);
    uint8_t *const dw = dst + 4ull * WB;  // (uniform)
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
    if (first && lane < EC_M) img[lane] = 0u;  // the bytes before A
    if (tl) pdb[tail_l - base] = 0u;
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

// ---------------------------------------------------------------------------
// decode: canonical multi-symbol decoder
// ---------------------------------------------------------------------------
#define HD_COUNT_ROW(LEN, LIM, FIRST, BASE) +1
enum {  // code lengths longer than the lookup (14-bit primary set, 13-bit set)
  NLONG = 0 HD_HUFF_LONG_CODES(HD_COUNT_ROW),
  NLONG13 = 0 HD_HUFF_LONG_CODES13(HD_COUNT_ROW)
};
#undef HD_COUNT_ROW

#define NLONG_PAD 16  // search width (padding rows repeat the last row)
static_assert(NLONG <= NLONG_PAD && NLONG13 <= NLONG_PAD, "long-code search too narrow");
// Lookup entry (tools/gen_tables.py): sym1 | sym2 << 8 | 8 cnt << 16 | L1 << 21 | used << 27
// (sym2 = 0 when cnt = 1: the low half is the entry's output bytes as they stand)
#define E_CNT8(e) (((e) >> 16) & 0x18u)
#define E_CNT(e) (((e) >> 19) & 3u)
#define E_L1(e) (((e) >> 21) & 31u)
#define E_USED(e) ((e) >> 27)
// The decoder's LDS tables for an LB-bit first-level lookup (14: 64 KB, the
// most two-symbol entries; 13: 32 KB, which leaves room for more waves).
template <int LB>
struct DecT {
  static constexpr int BITS = LB;
  static constexpr uint32_t NL = LB == 13 ? (uint32_t)NLONG13 : (uint32_t)NLONG;
  uint32_t lut[1 << LB];
  uint32_t lut2[64];               // codes of LB+1..16 bits (second level)
  uint32_t long_lim[NLONG_PAD];    // exclusive left-justified limit (last: ~0)
  uint32_t long_delta[NLONG_PAD];  // canonical base - first code (mod 2^32)
  uint32_t long_len[NLONG_PAD];
  uint16_t canon[260];
  uint32_t depth_lo[30];
  uint16_t depth_base[30];
  uint8_t depth_ids[256];
};
static_assert(HD_HUFF_LUT_BITS == 14, "primary lookup");
typedef DecT<HD_HUFF_LUT_BITS> DecTables;

template <int LB>
__device__ __forceinline__ void stage_dec_tables(DecT<LB> &T, uint32_t nthreads) {
  static_assert(LB == 13 || LB == 14, "lookup widths generated");
  const uint32_t t = threadIdx.x;
  const uint32_t *lut = LB == 13 ? dev::hd_huff_lut13 : dev::hd_huff_lut;
  const uint32_t *lut2 = LB == 13 ? dev::hd_huff_lut2_13 : dev::hd_huff_lut2;
  for (uint32_t i = t; i < (1u << LB); i += nthreads) T.lut[i] = lut[i];
  if (t < 64) T.lut2[t] = lut2[t];
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
    if (LB == 13) {
      HD_HUFF_LONG_CODES13(HD_LONG_ROW)
    } else {
      HD_HUFF_LONG_CODES(HD_LONG_ROW)
    }
#undef HD_LONG_ROW
    for (; i < NLONG_PAD; ++i) {
      T.long_lim[i] = 0xFFFFFFFFu;
      T.long_delta[i] = T.long_delta[DecT<LB>::NL - 1];
      T.long_len[i] = T.long_len[DecT<LB>::NL - 1];
    }
  }
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
#ifndef DEC_WAVES
#define DEC_WAVES 16  // waves per decode workgroup: one 64 KB lookup per CU
#endif
#define DEC_NT (WAVE * DEC_WAVES)
#define TASK_STR 64                                // strings per wave task
#ifndef PIECE_BYTES
// input bytes per item (string piece).  80 decodes config 3 in 558 us against
// 586 us isolated, but its 150 KB of LDS keeps encode workgroups off the CU
// in the 2-stream bench (900 vs 906 GB/s, tools/diag/ab_bench.sh)
#define PIECE_BYTES 64u
#endif
#ifndef SUB_OV
#define SUB_OV 24u                                 // warm-up bytes of a k > 0 piece
#endif
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
// bits 0..7 of v, sym2 in bits 8..15 (zero when c8 = 8).  Output goes straight
// to global memory: DwordSink for items that start an engine slot (dword
// aligned), UDwordSink for pieces that continue a string (their first byte
// may share a dword with the previous piece, another lane).
//
// Direct global output of an item that starts on a dword boundary: whole
// dwords from a 64-bit accumulator holding nb pending bits.  finish(): the
// string's last item may write its final dword whole (the slot is a dword
// multiple and holds more than the decoded bytes); otherwise the tail goes
// bytewise, since the next piece (another lane) continues in that dword.
struct DwordSink {
  uint32_t *p, *p0;
  uint64_t acc;
  uint32_t nb;
  __device__ __forceinline__ void init(uint8_t *q) {
    p = p0 = reinterpret_cast<uint32_t *>(q);
    acc = 0;
    nb = 0;
  }
  __device__ __forceinline__ uint32_t count() const { return 4u * (uint32_t)(p - p0) + (nb >> 3); }
  // put_nf: append without flushing (nb <= 31 before, so two of them fit)
  __device__ __forceinline__ void put_nf(uint32_t v, uint32_t c8) {
    acc |= (uint64_t)v << nb;
    nb += c8;
  }
  __device__ __forceinline__ void flush() {
#if HD_FLUSH_NOBRANCH
    // the pending low dword goes out every time (a partial one is rewritten
    // later, by this sink or by the next piece's head bytes)
    *p = (uint32_t)acc;
    const bool f = nb >= 32u;
    p += f ? 1 : 0;
    acc = f ? acc >> 32 : acc;
    nb -= f ? 32u : 0u;
#else
    if (nb >= 32u) {
      *p++ = (uint32_t)acc;
      acc >>= 32;
      nb -= 32u;
    }
#endif
  }
  __device__ __forceinline__ void put(uint32_t v, uint32_t c8) {
    put_nf(v, c8);
    flush();
  }
  __device__ __forceinline__ void finish(bool whole) {
    if (nb == 0) return;
    if (whole) {
      *p = (uint32_t)acc;
    } else {
      uint8_t *b = reinterpret_cast<uint8_t *>(p);
      for (uint32_t x = 0; x < (nb >> 3); ++x) b[x] = (uint8_t)(acc >> (8u * x));
    }
  }
};
// Direct global output of a piece that continues a string: the head dword
// (shared with the previous piece) goes bytewise, every later complete dword
// whole, and the tail as DwordSink::finish.
struct UDwordSink {
  uint32_t *p;
  uint64_t acc;
  uint32_t nb, n8, h;
  __device__ __forceinline__ void init(uint8_t *q) {
    h = (uint32_t)(uintptr_t)q & 3u;
    p = reinterpret_cast<uint32_t *>(q - h);
    acc = 0;
    nb = 8u * h;
    n8 = 0;
  }
  __device__ __forceinline__ uint32_t count() const { return n8 >> 3; }
  __device__ __forceinline__ void put_nf(uint32_t v, uint32_t c8) {
    acc |= (uint64_t)v << nb;
    nb += c8;
    n8 += c8;
  }
  __device__ __forceinline__ void put(uint32_t v, uint32_t c8) {
    put_nf(v, c8);
    flush();
  }
  __device__ __forceinline__ void flush() {
    if (nb >= 32u) {
      if (h) {  // the head dword: only bytes h..3 are this piece's
        uint8_t *b = reinterpret_cast<uint8_t *>(p);
        for (uint32_t x = h; x < 4u; ++x) b[x] = (uint8_t)(acc >> (8u * x));
        h = 0;
      } else {
        *p = (uint32_t)acc;
      }
      ++p;
      acc >>= 32;
      nb -= 32u;
    }
  }
  __device__ __forceinline__ void finish(bool whole) {
    const uint32_t na = nb >> 3;
    if (na <= h) return;
    if (whole && h == 0) {
      *p = (uint32_t)acc;
    } else {
      uint8_t *b = reinterpret_cast<uint8_t *>(p);
      for (uint32_t x = h; x < na; ++x) b[x] = (uint8_t)(acc >> (8u * x));
    }
  }
};
struct NullSink {
  uint32_t n8 = 0;
  __device__ __forceinline__ uint32_t count() const { return n8 >> 3; }
  __device__ __forceinline__ void put(uint32_t, uint32_t c8) { n8 += c8; }
  __device__ __forceinline__ void put_nf(uint32_t, uint32_t c8) { n8 += c8; }
  __device__ __forceinline__ void put2(uint32_t e1, uint32_t e2) { n8 += E_CNT8(e1) + E_CNT8(e2); }
  __device__ __forceinline__ void flush() {}
};
// Caller slots (any alignment, capacity checked), dword stores: as
// UDwordSink, with every store limited to the slot end `lim`; a byte at or
// past it is not written and marks the overflow.
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
    acc |= (uint64_t)v << nb;
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

// Code longer than the lookup: canonical length by a branch-free search over
// the left-justified limits (one row per code length, padded to 16 rows),
// then the symbol.  Returns a lookup-style entry
// (cnt 1, used = L), or ~0u when EOS (symbol 256) completes within `rem`.
template <class TT>
__device__ __forceinline__ uint32_t long_entry(const TT &T, uint32_t win, uint32_t rem) {
  uint32_t i = 0;
#pragma unroll
  for (uint32_t step = NLONG_PAD / 2; step; step >>= 1)
    i += (T.long_lim[i + step - 1] <= win) ? step : 0u;
  i = min(i, TT::NL - 1u);  // win == ~0: the 30-bit row
  const uint32_t L = T.long_len[i];
  const uint32_t sym = T.canon[(win >> (32 - L)) + T.long_delta[i]];
  if (L <= rem && sym == 256) return 0xFFFFFFFFu;
  return (L <= rem ? sym : 0u) | (8u << 16) | (L << 21) | (L << 27);
}

// First-level miss: the second level (codes of up to 16 bits), else the search.
template <class TT>
__device__ __forceinline__ uint32_t slow_entry(const TT &T, uint32_t win, uint32_t rem) {
  const uint32_t e = T.lut2[(win >> 16) & 63u];
  return e ? e : long_entry(T, win, rem);
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
    sink.put_nf(e & 0xFFFFu, E_CNT8(e));                         \
    q += E_USED(e);                                              \
  } while (0)
  while ((int32_t)q < F2) {
    DCTR(0);
    DEC_FAST_STEP();
    DEC_FAST_STEP();
    sink.flush();
  }
  while ((int32_t)q < F) {
    DCTR(0);
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
    DCTR(1);
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
    sink.put(two ? e & 0xFFFFu : e & 0xFFu, two ? 16u : 8u);
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
// AUTO: engine slots (written to dst_off); else caller slots,
// capacity-checked.
struct DecShared {
  DecTables T;  // first: the lookup sits at LDS offset 0 (its base folds into ds_read's offset)
  uint32_t ibe[DEC_WAVES][IBUF_W / 4 + 4];  // per wave: 16 spare bytes, then the round's input
};

template <bool AUTO>
__global__ __launch_bounds__(DEC_NT) void k_decode(const uint8_t *__restrict__ src,
                                                   const uint32_t *__restrict__ off, uint32_t n,
                                                   uint8_t *__restrict__ dst, uint64_t dst_cap,
                                                   uint32_t *__restrict__ dst_off,
                                                   int32_t *__restrict__ status,
                                                   uint16_t *__restrict__ fstate_out,
                                                   uint8_t *__restrict__ flags_out) {
  __shared__ DecShared S;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  lds_u32 *ibw = (lds_u32 *)S.ibe[wv];
  const lds_u32 *ibe = ibw;
  stage_dec_tables(S.T, DEC_NT);  // the kernel's only workgroup barrier
  WSTAMP_INIT();
  const uint32_t off0 = off[0];
  const uint32_t ntask = (n + TASK_STR - 1u) / TASK_STR;
  uint32_t dctr[4] = {0, 0, 0, 0};
  (void)dctr;
  for (uint32_t task = blockIdx.x * DEC_WAVES + wv; task < ntask; task += gridDim.x * DEC_WAVES) {
    const uint32_t t0 = task * TASK_STR;
    const uint32_t nstr = min(n - t0, (uint32_t)TASK_STR);
    WCOUNT(8);
    // lane l: task string l
    const bool sl = lane < nstr;
    const uint32_t a_l = sl ? off[t0 + lane] : 0u;
    const uint32_t b_l = sl ? off[t0 + lane + 1] : 0u;
    if (AUTO && sl) {  // saturated at dst_cap (< 2^32, checked by the host)
      dst_off[t0 + lane] = (uint32_t)min(auto_slot(a_l - off0, t0 + lane), dst_cap);
      if (t0 + lane == n - 1) dst_off[n] = (uint32_t)min(auto_slot(b_l - off0, n), dst_cap);
    }
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
      WCOUNT(9);
      WSTAMP(0);
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
      WSTAMP(1);
      // the carried exit is a bit position of the previous round's staging
      if (carry_exit < NOSPEC) carry_exit -= 8u * (IB - IB_prev);
      IB_prev = IB;
      const uint32_t j = t0 + it.i;
      const uint32_t bseg = 8u * (it.s - IBX);
      const uint32_t bend = 8u * (min(it.b, it.s + PIECE_BYTES + 32u) - IBX);
      const uint32_t bstop = it.last ? bend : 8u * (it.s + PIECE_BYTES - IBX);
      bool slot_ovf = false;  // AUTO: the string's slot is beyond dst_cap
      uint64_t o = 0;
      uint32_t cap = 0;
      if (valid) {
        if (AUTO) {
          o = auto_slot(it.a - off0, j);
          slot_ovf = auto_slot(it.b - off0, j + 1) > dst_cap;
        } else {
          o = dst_off[j];
          cap = dst_off[j + 1] - (uint32_t)o;
        }
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
          if (slot_ovf) {
            ovf = true;
          } else if (!AUTO) {
            CheckedDwordSink sk;
            sk.init(dst + o, cap);
            r = decode_item<false>(S.T, ibe, bseg, bseg, bstop, bend, sk, dctr);
            sk.finish();
            ovf = sk.ovf;
          } else {
            DwordSink sk;
            sk.init(dst + o);
            r = decode_item<false>(S.T, ibe, bseg, bseg, bstop, bend, sk, dctr);
            sk.finish(it.last);
          }
          if (it.last) {
            uint32_t fs = 0, fl = 0;
            status[j] = finish_string(S.T, r, r.cnt, ovf, &fs, &fl);
            if (fstate_out) fstate_out[j] = (uint16_t)fs;
            if (flags_out) flags_out[j] = (uint8_t)fl;
          }
        } else {
          NullSink nk;
          r = decode_item<true>(S.T, ibe, bseg - 8u * SUB_OV, bseg, bstop, bend, nk, dctr);
        }
      }
      WSTAMP(2);
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
            r = decode_item<false>(S.T, ibe, pred, bseg, bstop, bend, nk, dctr);
          }
        }
      }
      WSTAMP(3);
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
      WSTAMP(4);
      // ---- pass 2: k > 0 exact, at the string's running symbol count
      if (valid && it.k > 0) {
        const uint32_t soff = seg - r.cnt;
        const uint32_t e0 = r.entry;
        SubOut r2;
        r2.entry = r2.exit = XFAIL;
        r2.cnt = 0;
        r2.t = r2.win = 0;
        r2.at_end = false;
        bool ovf = AUTO && slot_ovf;
        if (e0 != XFAIL && !ovf) {
          if (!AUTO) {
            CheckedDwordSink sk;
            sk.init(dst + o + min(soff, cap), cap > soff ? cap - soff : 0u);
            r2 = decode_item<false>(S.T, ibe, e0, bseg, bstop, bend, sk, dctr);
            sk.finish();
            ovf = soff + r2.cnt > cap;  // this piece or an earlier one overflowed
          } else {
            UDwordSink sk;
            sk.init(dst + o + soff);
            r2 = decode_item<false>(S.T, ibe, e0, bseg, bstop, bend, sk, dctr);
            sk.finish(it.last);
          }
        } else if (!AUTO) {
          ovf = soff > cap;
        }
        if (it.last) {
          uint32_t fs = 0, fl = 0;
          status[j] = finish_string(S.T, r2, soff + r2.cnt, ovf, &fs, &fl);
          if (fstate_out) fstate_out[j] = (uint16_t)fs;
          if (flags_out) flags_out[j] = (uint8_t)fl;
        }
      }
      WSTAMP(5);
      // ---- carry the string running into the next round
      carry_exit = __builtin_amdgcn_readlane(r.exit, nv - 1u);
      carry_cnt = __builtin_amdgcn_readlane(seg, nv - 1u);
      // the next round overwrites the staged input
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      WSTAMP(6);
    }
  }
  WSTAMP_FLUSH();
}

// ---------------------------------------------------------------------------
// Dense decode (decode_batch_auto): byte-balanced pieces across string
// boundaries, output staged in LDS and written back to back.
// ---------------------------------------------------------------------------
// A wave owns a task of TASK_STR consecutive strings and walks their encoded
// bytes [A, Z) in rounds of 64 pieces of DD_P bytes, one piece per lane,
// whatever the string boundaries, so every lane of a round has the same
// amount of input.  Lane l's piece [s, e) holds:
//   seg0   the string running into it (if s is not a string start): entry
//          at the first codeword boundary >= 8 s (or the string's tail),
//          found by a warm-up decode from max(string start, s - DD_OV) --
//          exact when the warm-up starts at the string start, else
//          speculative and verified against the previous lane's exit
//          (mismatches are re-decoded from it, so the result is exact);
//   rest   every string starting in [s, e), decoded exactly from its start.
// A segment decodes to the first boundary >= 8 e or to its string's end.
// The string ending in a piece is finished by that piece's lane: the status
// of seg0's string needs the symbols of the lanes before (a segmented scan
// over lanes); the others are complete in the lane.
// Symbols go to the lane's LDS output region, seg0 first; after the round
// a plain scan of the lanes' byte counts places every region at the task's
// running output count and each lane stores its bytes (dword stores, the
// unaligned ends bytewise).  The task's output is dense from its base
// auto_slot(x_t0, t0): string j at dst_off[j], the strings of a task back to
// back, so HBM sees the decoded bytes once (no slot gaps).
#ifndef DD_P
#define DD_P 32u   // piece bytes per lane
#endif
#ifndef DD_OV
#define DD_OV 20u  // warm-up bytes of a later item (24 before: 314.2 vs 306.5 us on config 3)
#endif
#ifndef DD_WAVES
#define DD_WAVES 14  // waves per workgroup: one lookup table per CU
#endif
#ifndef DD_SKEW
#define DD_SKEW 0  // staged input: a copy of the next block's first dword after every 8
#endif
#ifndef DD_ABL_NOSTORE
#define DD_ABL_NOSTORE 0  // ablation build only (tools/diag): no output stores
#endif
#ifndef DD_BB
#define DD_BB 1  // fast steps from a register bit buffer (else LDS windows)
#endif
#ifndef DD_BALANCE
#define DD_BALANCE 1  // item decoder (40-byte pieces): weight-balanced task ranges per workgroup
#endif
#ifndef DD_TASK_W
#define DD_TASK_W 32u  // item decoder: a string's weight in bytes when balancing tasks
#endif
#ifndef DD_CLAIM
#define DD_CLAIM 1  // item decoder: waves of a workgroup claim tasks from an LDS counter
#endif
#ifndef DD_CAREFUL2
#define DD_CAREFUL2 1  // careful steps as selects (every lane steps), not exec-mask branches
#endif
#ifndef DD_GIN
#define DD_GIN 0  // A/B builds: item decoders read their input through the caches, not LDS
#endif
#ifndef DD_XINST
#define DD_XINST 0  // A/B builds: more item-decoder instances (decode_batch_items piece 65/41/57/37)
#endif
#ifndef DD_CSTORE
#define DD_CSTORE 1  // item decoder, 64-byte items (2: all): a round's output compacted in
                     // LDS, then coalesced stores (measured slower with 40-byte items)
#endif
#ifndef DD_WSYNC
#define DD_WSYNC 1  // warm-ups end with boundary-only single steps (no careful steps)
#endif
#ifndef DD_W16
#define DD_W16 0  // a step's two symbol bytes as one unaligned ds_write_b16
#endif
#ifndef DD_LATE
#define DD_LATE 0  // item decoder: the next round's input staged at the end of a round (see kLate)
#endif
#ifndef DD_ST4
#define DD_ST4 1  // item decoder, realigned stores: four whole dwords as one 16-byte store
#endif
#ifndef DD_NTL
#define DD_NTL 0  // item decoder: the staged input read with nontemporal loads
#endif
#ifndef DD_NTS
#define DD_NTS 0  // item decoder: 16-byte output stores nontemporal
#endif
#ifndef DD_PICK_LONG
#define DD_PICK_LONG 40  // A/B builds: the instance decode_batch_auto picks for long strings
#endif
#ifndef DD_TAILPOST
#define DD_TAILPOST 0  // careful steps: the tail's bits and window taken after the loop
#endif
#ifndef DD_WMERGE
#define DD_WMERGE 0  // item decoder (with DD_MERGE): the warm-up through the same inlined decoder
#endif
#ifndef DD_MERGE
#define DD_MERGE 1  // item decoder: the item's decode and its re-decodes share one inlined copy
                    // (instances without a budget: those whose later pieces warm up)
#endif
#ifndef DD_CKPT
#define DD_CKPT 0  // item decoder: a missed warm-up entry re-decoded only up to a checkpoint
#endif
#ifndef DD_CKB
#define DD_CKB 48  // checkpoint distance (bits past a later item's entry)
#endif
#ifndef DD_HT2
#define DD_HT2 0  // item decoder, realigned stores: head and tail bytes as 2-byte stores
#endif
#ifndef DD_G2OLD
#define DD_G2OLD 0  // A/B builds: the round-2 fast-pair bound (bstop - 27, bend - 28)
#endif
#ifndef DD_WIN
#define DD_WIN 0  // fast pairs from a window read per pair (else a refilled register buffer)
#endif
#ifndef DD_WINC
#define DD_WINC 0  // careful steps: the window read per step (else the register buffer)
#endif
#ifndef DD_SLOWU
#define DD_SLOWU 0  // fast pairs: the long-code path behind a uniform (ballot) branch
#endif
#ifndef DD_ACC
#define DD_ACC 0  // item decoder: symbols gathered in a register word, one ds_write_b32 per pair
#endif
#define DD_NT (WAVE * DD_WAVES)
// a lane decodes bits [8 s, 8 e + 29] at most: <= (8 P + 29) / 5 symbols,
// plus one byte of slack (the second byte of a 1-symbol entry is written)
#define DD_RB ((((8u * DD_P + 29u) / 5u) + 2u + 3u) & ~3u)
#define DD_IBL ((WAVE * DD_P + DD_OV + 64u) / 4u + 8u)          // staged dwords (logical)
#define DD_PF ((WAVE * DD_P + DD_OV + 8u + 32u + 16u * WAVE - 1u) / (16u * WAVE))  // staged chunks per lane
#define DD_IBW (DD_SKEW ? DD_IBL + DD_IBL / 8u + 2u : DD_IBL)   // physical

struct DDShared {
  DecTables T;  // first: the lookup at LDS offset 0
  uint32_t ib[DD_WAVES][DD_IBW];
  uint32_t ob[DD_WAVES][WAVE * DD_RB / 4 + 1];
  uint32_t ostart[DD_WAVES][TASK_STR];  // string output starts (task-relative)
  uint32_t sa[DD_WAVES][TASK_STR + 1];  // the task's string starts, then its end Z
};

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
  uint32_t ostart[IW][TASK_STR];  // string output starts (task-relative)
  uint32_t smap[IW][WAVE];        // a round's items -> strings (1-based, max-scanned)
  uint32_t claimed;               // tasks of the workgroup's range claimed so far
};

struct DiscardSink {  // a warm-up: its symbols belong to the item before
  __device__ __forceinline__ uint32_t count() const { return 0; }
  __device__ __forceinline__ void put_nf(uint32_t, uint32_t) {}
  __device__ __forceinline__ void put2(uint32_t, uint32_t) {}
  __device__ __forceinline__ void put(uint32_t, uint32_t) {}
  __device__ __forceinline__ void flush() {}
};

// The item decoder's sink (DD_ACC): the lane's pending output bytes in a
// register word `lo` (na bits, < 32), written whole to the lane's LDS
// region with one ds_write_b32 per fast pair (up to four symbols) instead of
// two ds_write_b8 per step -- the pair loop is LDS-issue heavy (two gathered
// lookups, the input word, and before this four byte stores per pair).  The
// word is written at every put, so the region always holds the bytes so far
// (the bytes past count() are don't-care); a put that fills the word moves
// on to the next one with the bits that overflowed it.
struct LdsAccSink {
  lds_u32 *p, *base;
  uint32_t lo, na;
  __device__ __forceinline__ LdsAccSink(lds_u8 *b) : p((lds_u32 *)b), base((lds_u32 *)b), lo(0), na(0) {}
  __device__ __forceinline__ uint32_t count() const { return 4u * (uint32_t)(p - base) + (na >> 3); }
  // the two lookup entries of a fast pair (sym1 | sym2 << 8, 8 cnt at bits 16..20)
  __device__ __forceinline__ void put2(uint32_t e1, uint32_t e2) {
    const uint32_t c1 = E_CNT8(e1), c2 = E_CNT8(e2);
    const uint32_t v = ((e2 & 0xFFFFu) << c1) | (e1 & 0xFFFFu);  // <= 32 bits
    const uint64_t t = (uint64_t)v << na;
    lo |= (uint32_t)t;
    *p = lo;
    na += c1 + c2;
    const bool sp = na >= 32u;
    lo = sp ? (uint32_t)(t >> 32) : lo;
    p += sp ? 1 : 0;
    na &= 31u;
  }
  // one step's symbols: v holds c8 / 8 (0..2) bytes, nothing above them
  __device__ __forceinline__ void put(uint32_t v, uint32_t c8) {
    const uint64_t t = (uint64_t)v << na;
    lo |= (uint32_t)t;
    *p = lo;
    na += c8;
    const bool sp = na >= 32u;
    lo = sp ? (uint32_t)(t >> 32) : lo;
    p += sp ? 1 : 0;
    na &= 31u;
  }
  __device__ __forceinline__ void put_nf(uint32_t v, uint32_t c8) { put(v & 0xFFFFu, c8); }
  __device__ __forceinline__ void flush() { *p = lo; }
};

struct LdsSink {
  lds_u8 *p;
  uint32_t n;
  __device__ __forceinline__ uint32_t count() const { return n; }
  __device__ __forceinline__ void put_nf(uint32_t v, uint32_t c8) {
    if (DD_W16) {
      const uint32_t a = (uint32_t)(uintptr_t)(p + n);
      asm volatile("ds_write_b16 %0, %1" ::"v"(a), "v"(v));
    } else {
      p[n] = (uint8_t)v;
      p[n + 1] = (uint8_t)(v >> 8);
    }
    n += c8 >> 3;
  }
  __device__ __forceinline__ void put2(uint32_t e1, uint32_t e2) {
    put_nf(e1 & 0xFFFFu, E_CNT8(e1));
    put_nf(e2 & 0xFFFFu, E_CNT8(e2));
  }
  __device__ __forceinline__ void put(uint32_t v, uint32_t c8) { put_nf(v, c8); }
  __device__ __forceinline__ void flush() {}
};

// The item decoder's sink: a running LDS pointer (one add per step fewer
// than base + count).
struct LdsPtrSink {
  lds_u8 *p, *base;
  __device__ __forceinline__ LdsPtrSink(lds_u8 *b) : p(b), base(b) {}
  __device__ __forceinline__ uint32_t count() const { return (uint32_t)(p - base); }
  __device__ __forceinline__ void put_nf(uint32_t v, uint32_t c8) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p += c8 >> 3;
  }
  __device__ __forceinline__ void put2(uint32_t e1, uint32_t e2) {
    put_nf(e1 & 0xFFFFu, E_CNT8(e1));
    put_nf(e2 & 0xFFFFu, E_CNT8(e2));
  }
  __device__ __forceinline__ void put(uint32_t v, uint32_t c8) { put_nf(v, c8); }
  __device__ __forceinline__ void flush() {}
};
typedef std::conditional<DD_ACC != 0, LdsAccSink, LdsPtrSink>::type DISink;
static_assert(!(DD_CKPT && DD_ACC), "the checkpoint fix-up assumes the byte sink");

// the item decoder's 16-byte input loads and output stores (read or written
// once: optionally with the nontemporal hint)
__device__ __forceinline__ uint4 dd_ld16(const uint4 *p) {
  if (DD_NTL) {
    uint4 v;
    v.x = __builtin_nontemporal_load(&p->x);
    v.y = __builtin_nontemporal_load(&p->y);
    v.z = __builtin_nontemporal_load(&p->z);
    v.w = __builtin_nontemporal_load(&p->w);
    return v;
  }
  return *p;
}
__device__ __forceinline__ void dd_st16(uint4 *p, uint4 v) {
  if (DD_NTS) {
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
    __builtin_nontemporal_store(v.z, &p->z);
    __builtin_nontemporal_store(v.w, &p->w);
  } else {
    *p = v;
  }
}

// Staged input, skewed: logical dword k lives at k + k / 8, and each block of
// 8 is followed by a copy of the next block's first dword, so the two dwords
// of a window are adjacent while the 64 lanes' pieces (8 dwords apart for
// 32-byte pieces) fall on different LDS banks.
__device__ __forceinline__ uint32_t dd_phys(uint32_t k) { return DD_SKEW ? k + (k >> 3) : k; }
__device__ __forceinline__ uint32_t dd_win(const lds_u32 *ib, uint32_t q) {  // q = bp - 1
  const uint32_t p = dd_phys(q >> 5);
  return __builtin_amdgcn_alignbit(ib[p], ib[p + 1], ~q);
}

// Input word k (big-endian) of a decode: the wave's staged LDS copy, or the
// pool itself through the vector caches (DD_GIN A/B builds).
struct LdsIn {
  const lds_u32 *ib;
  __device__ __forceinline__ uint32_t operator()(uint32_t k) const { return ib[dd_phys(k)]; }
};
struct GlobalIn {
  const uint8_t *base;  // byte of word 0
  __device__ __forceinline__ uint32_t operator()(uint32_t k) const {
    return __builtin_bswap32(*reinterpret_cast<const uint32_t *>(base + 4u * k));
  }
};

struct DDRun {
  bool failed, at_end;
  uint32_t t, win;  // at the string end: tail bits and the last window
};

// Decode from bp (advanced in place) to the first codeword boundary >=
// bstop, or to the string end bend (tail analysis), into sink.
//
// Fast steps come from a register bit buffer: bb holds the stream's bits
// [bp, 32 k) MSB first (nb of them, >= 32 at a step's start), refilled
// without a branch from the staged dword k (prefetched in nxt), so a step's
// only dependent memory access is its lookup.  A fast step needs its 14
// lookup bits inside the string (bp + 14 <= bend) and must not pass the
// first boundary >= bstop (bp <= bstop - 13: the first symbol of a 2-symbol
// entry is <= 9 bits); pairs run while both steps qualify.  A code longer
// than the lookup (entry 0) stalls the lane for the rest of the pair, then
// goes through slow_entry; one that would pass the string end is its tail
// and leaves the fast loop.  The last bits go through checked steps (LDS
// windows), which also settle the tail: the undecoded t < 30 bits.
#define DD_REFILL()                                                      \
  do {                                                                   \
    const bool t_ = nb < 32u;                                            \
    bb |= (uint64_t)(t_ ? nxt : 0u) << ((32u - nb) & 63u);               \
    nb += t_ ? 32u : 0u;                                                 \
    k += t_ ? 1u : 0u;                                                   \
    nxt = ib(k);                                                         \
  } while (0)
// PAIRS: only the fast pairs, none starting past `lim` (no careful steps):
// bp stops at a codeword boundary on the way, for a caller that records it
// and goes on with another dd_run.
template <class Sink, bool SYNC = false, bool PAIRS = false, class TT, class IN>
__device__ __forceinline__ DDRun dd_run(const TT &T, const IN &ib, uint32_t &bp,
                                        uint32_t bstop, uint32_t bend, Sink &sink,
                                        uint32_t *dctr DD_SARGS, int32_t lim = INT32_MAX) {
  (void)dctr;
  WSTAMP(2);  // (the caller's bookkeeping)
  DDRun r;
  r.at_end = false;
  r.t = 0;
  r.win = 0;
  bool failed = false;
  // last start of a fast pair: every code it takes starts before bstop (the
  // second step's second symbol at most LB + (LB - 5) bits on) and ends
  // inside the string (two steps take at most 2 LB bits)
  int32_t G2 = DD_G2OLD ? min((int32_t)bstop - 27, (int32_t)bend - 28)
                        : min((int32_t)bstop - (2 * TT::BITS - 4), (int32_t)bend - 2 * TT::BITS);
  if (PAIRS) G2 = min(G2, lim);
  if (DD_WIN) {
    // fast pairs from a 32-bit window read at each pair's start (two staged
    // words and one v_alignbit: q = bp - 1, the window is {w[q/32],
    // w[q/32+1]} >> (~q & 31)) instead of a refilled 64-bit register buffer:
    // fewer VALU per pair, one more LDS read on the pair's chain
    uint32_t q = bp - 1u;
    const int32_t Gq = G2 - 1;
    while ((int32_t)q <= Gq) {
      DCTR(0);
      const uint32_t kq = q >> 5;
      const uint32_t win = __builtin_amdgcn_alignbit(ib(kq), ib(kq + 1u), ~q);
      const uint32_t e1 = T.lut[win >> (32 - TT::BITS)];
      const uint32_t U1 = E_USED(e1);
      const uint32_t e2 = T.lut[(win << U1) >> (32 - TT::BITS)];
      sink.put2(e1, e2);
      q += U1 + E_USED(e2);
      if (e2 == 0u) {  // a code longer than the lookup at q + 1 (an e1 of 0 stalls e2 too)
        const uint32_t kq2 = q >> 5;
        const uint32_t w = __builtin_amdgcn_alignbit(ib(kq2), ib(kq2 + 1u), ~q);
        const uint32_t rem_ = bend - (q + 1u);
        const uint32_t e_ = slow_entry(T, w, rem_);
        if (e_ == 0xFFFFFFFFu) {
          failed = true;
          break;
        } else if (E_L1(e_) > rem_) {
          break;  // the string's tail: the careful steps find it again
        }
        sink.put(e_ & 0xFFFFu, E_CNT8(e_));
        q += E_USED(e_);
      }
    }
    bp = q + 1u;
    G2 = INT32_MIN;  // (the register-buffer loop below does not run)
  }
  uint32_t k = bp >> 5;
  const uint32_t o = bp & 31u;
  const uint32_t w0 = ib(k), w1 = ib(k + 1u);
  uint64_t bb = (((uint64_t)w0 << 32) | w1) << o;
  uint32_t nb = 64u - o;
  k += 2u;
  uint32_t nxt = ib(k);
  // a code longer than the lookup inside the pair loop (nb >= 32): decode
  // it, or leave the pair loop at EOS (failed) or at the string's tail
  // (the careful steps find it again)
#define DD_SLOW()                                                        \
  do {                                                                   \
    const uint32_t rem_ = bend - bp;                                     \
    const uint32_t e_ = slow_entry(T, (uint32_t)(bb >> 32), rem_);       \
    if (e_ == 0xFFFFFFFFu) {                                             \
      failed = true;                                                     \
      G2 = INT32_MIN;                                                    \
    } else if (E_L1(e_) > rem_) {                                        \
      G2 = INT32_MIN;                                                    \
    } else {                                                             \
      sink.put(e_ & 0xFFFFu, E_CNT8(e_));                                \
      const uint32_t U_ = E_USED(e_);                                    \
      bb <<= U_;                                                         \
      bp += U_;                                                          \
      nb -= U_;                                                          \
      DD_REFILL();                                                       \
    }                                                                    \
  } while (0)
  while ((int32_t)bp <= G2) {
    DCTR(0);
    const uint32_t e1 = T.lut[(uint32_t)(bb >> 32) >> (32 - TT::BITS)];
    const uint32_t U1 = E_USED(e1);
    bb <<= U1;
    const uint32_t e2 = T.lut[(uint32_t)(bb >> 32) >> (32 - TT::BITS)];
    sink.put2(e1, e2);
    const uint32_t U2 = E_USED(e2);
    bb <<= U2;
    bp += U1 + U2;
    nb -= U1 + U2;
    DD_REFILL();
    if (DD_SLOWU) {  // the rare long code behind one uniform branch
      if (__ballot(e2 == 0u)) {
        if (e2 == 0u) DD_SLOW();
      }
    } else if (e2 == 0u) {
      DD_SLOW();  // (an e1 of 0 stalls e2 too)
    }
  }
#undef DD_SLOW
  WSTAMP(10);
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
    bool done = failed || (int32_t)bp >= (int32_t)bstop;
    while (__ballot(!done)) {
      if (!done) {
        DCTR(2);
        const uint32_t w = (uint32_t)(bb >> 32);
        uint32_t e = T.lut[w >> (32 - TT::BITS)];
        if (e == 0u) e = slow_entry(T, w, 30u);
        const uint32_t L1 = E_L1(e), adv = bp + L1 >= bstop ? L1 : E_USED(e);
        if (e == 0xFFFFFFFFu || bp + adv > bend) {
          failed = true;
          done = true;
        } else {
          bb <<= adv;
          bp += adv;
          nb -= adv;
          DD_REFILL();
          done = bp >= bstop;
        }
      }
    }
    r.failed = failed;
    return r;
  }
  // careful steps: each one predicated on the stop rules instead of branching
  // -- a step takes its first symbol only if the code ends inside the string
  // (L1 <= rem), its second only if that one does too and the first ended
  // before bstop; a first code that does not fit is the string's tail
  bool done = failed;
  if (DD_CAREFUL2) {
    // the same steps with every lane stepping (a finished lane takes
    // nothing): selects instead of exec-mask branches, the rare long code
    // behind one uniform branch
    while (__ballot(!done)) {
      DCTR(2);
      // (DD_WINC: the step's window read from the staged words at bp)
      const uint32_t w = DD_WINC ? __builtin_amdgcn_alignbit(ib((bp - 1u) >> 5), ib(((bp - 1u) >> 5) + 1u), ~(bp - 1u))
                                 : (uint32_t)(bb >> 32);
      const uint32_t rem = bend - bp;
      const bool stop = done || bp >= bstop || rem == 0u;
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
      r.at_end = r.at_end || tail;
      if (!DD_TAILPOST) {
        r.t = tail ? rem : r.t;
        r.win = tail ? w : r.win;
      }
      const uint32_t adv = take2 ? U : (take1 ? L1 : 0u);
      sink.put(take2 ? (e & 0xFFFFu) : (take1 ? (e & 0xFFu) : 0u), take2 ? 16u : (take1 ? 8u : 0u));
      bp += adv;
      if (!DD_WINC) {
        bb <<= adv;
        nb -= adv;
        DD_REFILL();
      }
      failed = failed || eos;
      done = done || eos || !take1 || bp >= bstop;
    }
  }
  while (__ballot(!done)) {
    if (!done) {
      DCTR(2);
      const uint32_t w = (uint32_t)(bb >> 32);
      const uint32_t rem = bend - bp;
      const bool stop = bp >= bstop || rem == 0u;
      uint32_t e = T.lut[w >> (32 - TT::BITS)];
      if (e == 0u && !stop) e = slow_entry(T, w, rem);
      if (e == 0xFFFFFFFFu) {
        failed = true;  // EOS: the sticky failure state
        done = true;
      } else {
        const uint32_t L1 = E_L1(e), U = E_USED(e);
        const bool take1 = !stop && L1 <= rem;
        const bool take2 = take1 && E_CNT(e) == 2u && U <= rem && bp + L1 < bstop;
        if (!stop && !take1) {  // the tail: a proper prefix of a code
          r.at_end = true;
          r.t = rem;
          r.win = w;
        }
        const uint32_t adv = take2 ? U : (take1 ? L1 : 0u);
        sink.put(take2 ? (e & 0xFFFFu) : (take1 ? (e & 0xFFu) : 0u), take2 ? 16u : (take1 ? 8u : 0u));
        bb <<= adv;
        bp += adv;
        nb -= adv;
        DD_REFILL();
        done = !take1 || bp >= bstop;
      }
    }
  }
  if (DD_TAILPOST && DD_CAREFUL2 && !DD_WINC && r.at_end) {
    // the tail's bits and window, after the loop: a lane that met its tail
    // took no step after it (the refills only add stream bits below them)
    r.t = bend - bp;
    r.win = (uint32_t)(bb >> 32);
  }
  WSTAMP(11);
  sink.flush();
  if (!failed && bp == bend) r.at_end = true;
  r.failed = failed;
  WSTAMP(12);
  return r;
}
#undef DD_REFILL

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

#define DD_NONE 0xFFFFFFFCu  // exit: the lane's last string ended in its piece
enum { DD_WARM = 0, DD_SEG0 = 1, DD_REST = 2, DD_DONE = 3 };

__global__ __launch_bounds__(DD_NT) void k_decode_dense(const uint8_t *__restrict__ src,
                                                        const uint32_t *__restrict__ off,
                                                        uint32_t n, uint8_t *__restrict__ dst,
                                                        uint64_t dst_cap,
                                                        uint32_t *__restrict__ dst_off,
                                                        int32_t *__restrict__ status,
                                                        uint16_t *__restrict__ fstate_out,
                                                        uint8_t *__restrict__ flags_out) {
  __shared__ DDShared S;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  lds_u32 *ibw = (lds_u32 *)S.ib[wv];
  const lds_u32 *ibe = ibw;
  lds_u8 *my_ob = (lds_u8 *)S.ob[wv] + lane * DD_RB;
  const lds_u32 *my_ob32 = (const lds_u32 *)my_ob;
  lds_u32 *ost = (lds_u32 *)S.ostart[wv];
  lds_u32 *sa = (lds_u32 *)S.sa[wv];
  stage_dec_tables(S.T, DD_NT);  // the kernel's only workgroup barrier
  WSTAMP_INIT();
  const uint32_t off0 = off[0];
  const uint32_t ntask = (n + TASK_STR - 1u) / TASK_STR;
  uint32_t dctr[4] = {0, 0, 0, 0};
  (void)dctr;
  for (uint32_t task = blockIdx.x * DD_WAVES + wv; task < ntask; task += gridDim.x * DD_WAVES) {
    WCOUNT(8);
    const uint32_t t0 = task * TASK_STR;
    const uint32_t nstr = min(n - t0, (uint32_t)TASK_STR);
    const bool sl = lane < nstr;
    const uint32_t a_l = sl ? off[t0 + lane] : 0xFFFFFFFFu;
    const uint32_t b_l = sl ? off[t0 + lane + 1] : 0xFFFFFFFFu;
    const uint32_t A = __builtin_amdgcn_readfirstlane(a_l);
    const uint32_t Z = __builtin_amdgcn_readlane(b_l, nstr - 1u);
    const uint64_t tbase = auto_slot(A - off0, t0);
    // a string whose slot bound passes dst_cap reports -502 (monotone in j;
    // checked per string only in a task that reaches past dst_cap)
    const bool task_ovf = auto_slot(Z - off0, t0 + nstr) > dst_cap;
    const bool ovf_l = sl && task_ovf && auto_slot(b_l - off0, t0 + lane + 1u) > dst_cap;
    ost[lane] = 0xFFFFFFFFu;
    if (sl) sa[lane] = a_l;
    if (lane == 0) sa[nstr] = Z;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t carry_exit = DD_NONE, carry_cnt = 0, IB_prev = 0, run = 0;
    for (uint32_t R = A; R < Z; R += WAVE * DD_P) {
      const uint32_t s = R + lane * DD_P;
      const bool valid = s < Z;
      const uint32_t e = min(s + DD_P, Z);
      const uint32_t nv = min((Z - R + DD_P - 1u) / DD_P, (uint32_t)WAVE);
      // lb = the strings starting before s (task strings are contiguous and
      // ordered, empty ones included); string lb - 1 holds byte s when it
      // ends past s
      uint32_t lb = 0;
#pragma unroll
      for (uint32_t st = 32; st; st >>= 1)
        if (lb + st <= nstr && sa[lb + st - 1u] < s) lb += st;
      if (lb < nstr && sa[lb] < s) ++lb;
      const uint32_t j0 = lb ? lb - 1u : 0u;
      const uint32_t a0 = sa[j0], b0 = sa[j0 + 1u];
      const bool mid = valid && lb > 0 && b0 > s;  // the piece starts inside string j0
      WCOUNT(9);
      WSTAMP(0);
      // ---- stage [max(A, R - OV), min(R + 64 P, Z) + 8) (aligned 16-byte chunks)
      const uint32_t lo = (R - A > DD_OV ? R - DD_OV : A);
      const uint32_t IB = lo & ~15u;
      const uint32_t IBX = IB - 16u;
      {
        const uint32_t hi = min(R + WAVE * DD_P, Z) + 8u;
        const uint32_t nchunk = (((hi + 15u) & ~15u) - IB) >> 4;
        const uint4 *g = reinterpret_cast<const uint4 *>(src + IB);
        for (uint32_t c = lane; c < nchunk; c += WAVE) {
          const uint4 v = g[c];
          const uint32_t k = 4u * c + 4u;  // logical dword (4 spare dwords first)
          const uint32_t p = dd_phys(k);   // the chunk's 4 dwords stay in one block
          ibw[p] = __builtin_bswap32(v.x);
          ibw[p + 1] = __builtin_bswap32(v.y);
          ibw[p + 2] = __builtin_bswap32(v.z);
          ibw[p + 3] = __builtin_bswap32(v.w);
          if (DD_SKEW && (k & 7u) == 0u) ibw[p - 1] = __builtin_bswap32(v.x);  // the copy
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      WSTAMP(1);
      if (carry_exit < DD_NONE) carry_exit -= 8u * (IB - IB_prev);
      IB_prev = IB;
      const uint32_t bs = 8u * (s - IBX), bE = 8u * (e - IBX);
      // ---- one decode loop per lane over its piece: seg0's warm-up, seg0,
      // then the strings starting in the piece.  The wave runs the loop while
      // any lane has a segment left, so lanes in different segments share
      // the same decode steps.
      const bool fin0 = mid && b0 <= e;  // seg0's string ends in this piece
      const uint32_t bend0 = 8u * (min(b0, e + 8u) - IBX);
      const uint32_t bstop0 = fin0 ? bend0 : bE;
      const bool exact0 = !mid || a0 + DD_OV >= s;
      SubOut r0;
      r0.entry = r0.exit = DD_NONE;
      r0.cnt = 0;
      r0.t = r0.win = 0;
      r0.at_end = false;
      LdsSink sk;
      sk.p = my_ob;
      sk.n = 0;
      uint32_t mode = !valid ? DD_DONE : (mid ? DD_WARM : DD_REST);
      uint32_t bp = 0, bstop = 0, bend = 0;
      uint32_t j = lb, c_before = 0, cnt0 = 0;
      uint32_t tail_exit = DD_NONE, tail_cnt = 0;
      bool head = false;  // a string starts in this piece
      if (mode == DD_WARM) {
        bp = 8u * ((exact0 ? a0 : s - DD_OV) - IBX);
        bstop = bs;
        bend = bend0;
      }
      // next rest string: empty ones are finished on the spot
      auto next_string = [&]() {
        while (j < nstr && sa[j] < e) {
          const uint32_t a = sa[j], b = sa[j + 1u];
          head = true;
          ost[j] = sk.n - cnt0;  // relative to the rest's first byte (fixed after the scan)
          if (a != b) {
            bp = 8u * (a - IBX);
            bend = 8u * (min(b, e + 8u) - IBX);
            bstop = b <= e ? bend : bE;
            c_before = sk.n;
            mode = DD_REST;
            return;
          }
          dd_finish(S.T, false, 0, 0, 0, task_ovf && auto_slot(b - off0, t0 + j + 1u) > dst_cap,
                    t0 + j, status, fstate_out, flags_out);
          ++j;
        }
        mode = DD_DONE;
      };
      if (mode == DD_REST) next_string();
      while (__ballot(mode != DD_DONE)) {
        WCOUNT(6);
        if (mode != DD_DONE) {
          const DDRun rr = dd_run(S.T, LdsIn{ibe}, bp, bstop, bend, sk, dctr DD_SPASS);
          if (mode == DD_WARM) {
            // the entry: the first boundary >= 8 s, or the string's tail
            sk.n = 0;  // the warm-up's symbols belong to the lane before
            if (rr.failed) {  // EOS before s: known failed if exact
              r0.entry = r0.exit = exact0 ? XFAIL : XUNKNOWN;
              cnt0 = 0;
              j = lb;
              next_string();
            } else {
              r0.entry = bp;
              bstop = bstop0;
              mode = DD_SEG0;
            }
          } else if (mode == DD_SEG0) {
            r0.exit = rr.failed ? XFAIL : bp;
            r0.at_end = rr.at_end;
            r0.t = rr.t;
            r0.win = rr.win;
            cnt0 = sk.n;
            r0.cnt = cnt0;
            j = lb;
            next_string();
          } else {  // DD_REST: string j
            const uint32_t b = sa[j + 1u];
            if (b <= e) {  // it ends in this piece: finished
              dd_finish(S.T, rr.failed, rr.t, rr.win, sk.n - c_before,
                        task_ovf && auto_slot(b - off0, t0 + j + 1u) > dst_cap, t0 + j, status,
                        fstate_out, flags_out);
              tail_exit = DD_NONE;
              tail_cnt = 0;
              ++j;
              next_string();
            } else {  // it runs into the next piece: the lane's open tail
              tail_exit = rr.failed ? XFAIL : bp;
              tail_cnt = sk.n - c_before;
              ++j;
              mode = DD_DONE;
            }
          }
        }
      }
      const uint32_t jr1 = j;  // rest strings [lb, jr1)
      const uint32_t rest_n = sk.n - cnt0;
      WSTAMP(2);
      // ---- verify seg0 against the previous lane's exit; re-decode mismatches
      uint32_t my_exit = head ? tail_exit : (mid && !fin0 ? r0.exit : DD_NONE);
      uint32_t c0 = cnt0;
      for (uint32_t iter = 0; iter <= WAVE; ++iter) {
        // the previous lane's exit (wave_shr:1), lane 0 the carried one
        const uint32_t pred = (uint32_t)__builtin_amdgcn_update_dpp(
            (int)carry_exit, (int)my_exit, 0x138, 0xf, 0xf, false);
        const bool mism = mid && !exact0 && (r0.entry != pred || r0.entry == XUNKNOWN);
        const uint64_t bal = __ballot(mism);
        if (bal == 0) break;
        const bool pred_mism = lane && ((bal >> (lane - 1u)) & 1u);
        if (mism && !pred_mism) {
          // re-decode seg0 from the settled exit (a warm-up that did not
          // synchronise); the rest's bytes wait at the region's end meanwhile
          // (backward copy: the target lies past the source)
          for (uint32_t k = rest_n; k-- > 0;) my_ob[DD_RB - rest_n + k] = my_ob[c0 + k];
          LdsSink s3;
          s3.p = my_ob;
          s3.n = 0;
          if (pred == XFAIL || pred == XUNKNOWN || pred == DD_NONE) {
            r0.entry = r0.exit = XFAIL;  // the string failed before this piece
            r0.cnt = 0;
            r0.t = r0.win = 0;
            r0.at_end = false;
          } else {
            uint32_t bq = pred;
            const DDRun rr = dd_run(S.T, LdsIn{ibe}, bq, bstop0, bend0, s3, dctr DD_SPASS);
            r0.entry = pred;
            r0.exit = rr.failed ? XFAIL : bq;
            r0.t = rr.t;
            r0.win = rr.win;
            r0.at_end = rr.at_end;
            r0.cnt = s3.n;
          }
          for (uint32_t k = 0; k < rest_n; ++k) my_ob[s3.n + k] = my_ob[DD_RB - rest_n + k];
          c0 = s3.n;
          if (!head && !fin0) my_exit = r0.exit;
        }
      }
      WSTAMP(3);
      // ---- seg0's running symbol count: segmented scan over the lanes (heads:
      // pieces where a string starts); V = the count of the lane's open tail
      const uint32_t V = valid ? (head ? tail_cnt : c0) : 0u;
      const bool H = !valid || head;
      uint32_t ps = V;
      int32_t hm = H ? (int32_t)lane : -1;
#pragma unroll
      for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t o2 = __shfl_up(ps, d, 64);
        const int32_t oh = __shfl_up(hm, d, 64);
        if (lane >= d) {
          ps += o2;
          hm = max(hm, oh);
        }
      }
      const uint32_t excl_h = __shfl(ps - V, hm >= 0 ? (uint32_t)hm : 0u, 64);
      const uint32_t seg = hm >= 0 ? ps - excl_h : ps + carry_cnt;  // inclusive
      const uint32_t seg_prev_up = __shfl_up(seg, 1, 64);
      const uint32_t seg_prev = lane ? seg_prev_up : carry_cnt;
      if (fin0) {  // seg0's string ends here
        dd_finish(S.T, r0.exit == XFAIL || r0.entry == XFAIL, r0.t, r0.win, seg_prev + c0,
                  task_ovf && auto_slot(b0 - off0, t0 + j0 + 1u) > dst_cap, t0 + j0, status,
                  fstate_out, flags_out);
      }
      // ---- place the lanes' bytes: plain scan of the byte counts
      const uint32_t T_l = valid ? c0 + rest_n : 0u;
      const uint32_t Tinc = wave_incl_scan(T_l);
      const uint32_t O_l = run + Tinc - T_l;  // task-relative
      for (uint32_t jj = lb; jj < jr1; ++jj) ost[jj] += O_l + c0;
      WSTAMP(4);
      // ---- store [tbase + O_l, + T_l) from the region: the bytes before the
      // first aligned dword, then dwords (two region dwords, one alignbyte),
      // then the tail bytes; nothing at or past dst_cap is written (strings
      // past it are -502)
      if (T_l && !DD_ABL_NOSTORE) {
        const uint64_t g0 = tbase + O_l;
        const uint32_t h = min((uint32_t)((4u - (g0 & 3u)) & 3u), T_l);  // head bytes
        for (uint32_t k = 0; k < h; ++k)
          if (g0 + k < dst_cap) dst[g0 + k] = my_ob[k];
        uint32_t k = h;
        for (; k + 4u <= T_l; k += 4u) {
          const uint32_t w = k >> 2;
          const uint32_t v = __builtin_amdgcn_alignbyte(my_ob32[w + 1u], my_ob32[w], h);
          if (g0 + k + 4u <= dst_cap) *reinterpret_cast<uint32_t *>(dst + g0 + k) = v;
        }
        for (; k < T_l; ++k)
          if (g0 + k < dst_cap) dst[g0 + k] = my_ob[k];
      }
      WSTAMP(5);
      run += __builtin_amdgcn_readlane(Tinc, 63);
      carry_exit = __builtin_amdgcn_readlane(my_exit, nv - 1u);
      carry_cnt = __builtin_amdgcn_readlane(seg, nv - 1u);
      // the next round overwrites the staged input and the regions
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    // ---- epilogue: output starts (dst_off); empty strings at the task's end
    if (sl) {
      uint32_t o = ost[lane];
      if (o == 0xFFFFFFFFu) {  // an empty string at Z (or an all-empty task)
        o = run;
        dd_finish(S.T, false, 0, 0, 0, ovf_l, t0 + lane, status, fstate_out, flags_out);
      }
      dst_off[t0 + lane] = (uint32_t)min(tbase + o, dst_cap);
      if (t0 + lane == n - 1u) dst_off[n] = (uint32_t)min(tbase + run, dst_cap);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  WSTAMP_FLUSH_W(DD_WAVES);
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
template <uint32_t IP, int IW, int LB, uint32_t BI = 0>
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
  lds_u32 *ost = (lds_u32 *)S.ostart[wv];
  if (threadIdx.x == 0) S.claimed = 0u;
  stage_dec_tables(S.T, (WAVE * IW));  // the kernel's only workgroup barrier
  WSTAMP_INIT();
  const uint32_t off0 = off[0];
  const uint32_t ntask = (n + TASK_STR - 1u) / TASK_STR;
  uint32_t dctr[4] = {0, 0, 0, 0};
  (void)dctr;
  // this workgroup's tasks: with 40-byte pieces (long values, whose tasks
  // differ several-fold in work) a contiguous range balanced by weight
  // (encoded bytes + DD_TASK_W per string) over the grid, its waves striding
  // over it (config 3: 348 vs 356 us); else the grid strides over all tasks
  // (the search costs a short batch more than it saves)
  constexpr bool kBal = DD_BALANCE && IP == 40u;
  uint32_t t_lo, t_hi;
  {
    const uint32_t nwg = gridDim.x, g = blockIdx.x;
    const uint64_t wtot = (uint64_t)(off[n] - off0) + (uint64_t)DD_TASK_W * n;
    auto first_at = [&](uint64_t target) -> uint32_t {  // smallest t with weight(t) >= target
      if (target == 0) return 0u;
      uint32_t lo = 0, hi = ntask;  // weight(lo) < target <= weight(hi)
      while (hi - lo > 1u) {
        const uint32_t step = (hi - lo + WAVE - 1u) / WAVE;
        const uint32_t c = min(lo + (lane + 1u) * step, hi);
        const uint32_t sc = min(c * (uint32_t)TASK_STR, n);
        const uint64_t wc = (uint64_t)(off[sc] - off0) + (uint64_t)DD_TASK_W * sc;
        const uint64_t ge = __ballot(wc >= target);  // (lane 63 or the clamp reaches hi)
        const uint32_t j = ge ? (uint32_t)__builtin_ctzll(ge) : WAVE - 1u;
        const uint32_t nhi = __builtin_amdgcn_readlane(c, j);
        lo = j ? __builtin_amdgcn_readlane(c, j - 1u) : lo;
        hi = nhi;
      }
      return hi;
    };
    if (DD_CLAIM) {  // contiguous workgroup ranges (by weight or by count)
      t_lo = kBal ? first_at(wtot * g / nwg) : (uint32_t)((uint64_t)ntask * g / nwg);
      t_hi = g + 1u == nwg ? ntask
                           : kBal ? first_at(wtot * (g + 1u) / nwg)
                                  : (uint32_t)((uint64_t)ntask * (g + 1u) / nwg);
    } else {
      t_lo = kBal ? first_at(wtot * g / nwg) : g * IW;
      t_hi = kBal ? (g + 1u == nwg ? ntask : first_at(wtot * (g + 1u) / nwg)) : ntask;
    }
  }
  // DD_CLAIM: a wave's first task is t_lo + wv, later ones are claimed from
  // the workgroup's LDS counter one task ahead (so the waves of a CU finish
  // within a task of each other); else a fixed stride
  const uint32_t t_first = t_lo + wv, t_step = kBal ? (uint32_t)IW : gridDim.x * IW;
  auto claim_next = [&](uint32_t cur) -> uint32_t {
    if (!DD_CLAIM) return cur + t_step;
    uint32_t v = 0;
    if (lane == 0) v = atomicAdd((uint32_t *)&S.claimed, 1u);
    return t_lo + IW + __builtin_amdgcn_readfirstlane(v);
  };
  // a task's string offsets are loaded one task ahead (DD_LATE: two), and
  // the first round of the next task is staged into registers during the
  // current task's last round (pf), so neither waits at a task start
  uint32_t na_l = 0, nb_l = 0, n2a_l = 0, n2b_l = 0;
  auto load_offs = [&](uint32_t tk, uint32_t &xa, uint32_t &xb) {
    const uint32_t u0 = tk * TASK_STR;
    const bool in = tk < ntask && lane < min(n - u0, (uint32_t)TASK_STR);
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
  // DD_LATE: vmcnt counts loads and stores together and in order, so a wait
  // for loads issued after a round's output stores waits for those stores
  // too.  The prefetched input of the next round is therefore written to the
  // staging buffer at the END of the current round (after its verify, before
  // its status and output stores), and the string offsets are loaded two
  // tasks ahead and moved along at the end of a task (after that wait): every
  // wait then falls a whole round after the last stores.
  constexpr bool kLate = DD_LATE && !DD_GIN;
  uint4 pf[kPF];
  uint32_t pf_IB = 0xFFFFFFFFu, pf_n = 0, staged_IB = 0xFFFFFFFFu;
  uint32_t ca_l = 0, cb_l = 0;  // kLate: the current task's offsets
  load_offs(t_first < t_hi ? t_first : ntask, kLate ? ca_l : na_l, kLate ? cb_l : nb_l);
  uint32_t next_task = t_hi, next2 = t_hi;
  if (kLate) {
    next_task = t_first < t_hi ? claim_next(t_first) : t_hi;
    load_offs(next_task < t_hi ? next_task : ntask, na_l, nb_l);
    next2 = next_task < t_hi ? claim_next(next_task) : t_hi;
    __builtin_amdgcn_s_waitcnt(0x0F70);  // (the loop's first wait-free copies)
  }
  // kLate: the next task becomes the current one, the one after it the next
  // (after a round's wait; the offsets of the task after those are loaded at
  // the top of the task, so no register copy at the loop latch waits for them)
  auto rotate = [&]() {
    ca_l = na_l;
    cb_l = nb_l;
    na_l = n2a_l;
    nb_l = n2b_l;
    next_task = next2;
    next2 = next2 < t_hi ? claim_next(next2) : t_hi;
  };
  for (uint32_t task = t_first; task < t_hi;) {
    if (kLate) load_offs(next2 < t_hi ? next2 : ntask, n2a_l, n2b_l);
    else next_task = claim_next(task);
    WCOUNT(8);
    const uint32_t t0 = task * TASK_STR;
    const uint32_t nstr = min(n - t0, (uint32_t)TASK_STR);
    const bool sl = lane < nstr;
    const uint32_t a_l = kLate ? ca_l : na_l, b_l = kLate ? cb_l : nb_l;
    const uint32_t A = __builtin_amdgcn_readfirstlane(a_l);
    const uint32_t Z = __builtin_amdgcn_readlane(b_l, nstr - 1u);
    if (!kLate) load_offs(next_task < t_hi ? next_task : ntask, na_l, nb_l);
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
      staged_IB = 0xFFFFFFFFu;  // (staged for this task's first round)
      task = next_task;
      if (kLate) {
        __builtin_amdgcn_s_waitcnt(0x0F70);  // (as at a round's end)
        rotate();
      }
      continue;
    }
    // items: m_l of string l, X_l the first
    const uint32_t m_l = sl ? max(1u, (b_l - a_l + IP - 1u) / IP) : 0u;
    const uint32_t P_l = wave_incl_scan(m_l), X_l = P_l - m_l;
    const uint32_t M = __builtin_amdgcn_readlane(P_l, 63);
    uint32_t carry_exit = DD_NONE, carry_cnt = 0, IB_prev = 0, run = 0;
    uint32_t ocarry = 0;  // the partial last output word of the round before
    lds_u32 *smap = (lds_u32 *)S.smap[wv];
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
        smap[lane] = 0u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (sl && P_l > r0 && X_l < r0 + WAVE) smap[X_l > r0 ? X_l - r0 : 0u] = lane + 1u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        i = min(wave_incl_max(smap[lane]), nstr) - 1u;
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
        my_ob32 = (const lds_u32 *)my_ob;
      }
      const bool valid = lane < nv;
      const bool last = e == b;
      const bool spec = valid && k > 0;
      WCOUNT(9);
      WSTAMP(0);
      // ---- stage [first item (- OV), last item's end + 8)
      uint32_t IB, nchunk;
      round_range(R0, A, Z, IB, nchunk);
      const uint32_t IBX = IB - 16u;
#if DD_GIN
      const GlobalIn inp{src + IB - 16};
#else
      const LdsIn inp{ibe};
#endif
      // the prefetched chunks (pf) into the staging buffer, byte-swapped
      auto stage_pf = [&](uint32_t nch) {
#pragma unroll
        for (uint32_t u = 0; u < kPF; ++u) {
          const uint32_t c = lane + WAVE * u;
          if (c < nch) {
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
      if (!DD_GIN) {
        // (kLate: only a round that the round before did not stage)
        if (!kLate || staged_IB != IB) {
          const uint4 *g = reinterpret_cast<const uint4 *>(src + IB);
          if (pf_IB != IB) {  // (not prefetched)
#pragma unroll
            for (uint32_t u = 0; u < kPF; ++u)
              if (lane + WAVE * u < nchunk) pf[u] = dd_ld16(g + lane + WAVE * u);
          }
          stage_pf(nchunk);
        }
        // prefetch the next round: of this task, else the next task's first
        pf_IB = 0xFFFFFFFFu;
        uint32_t IBn = 0, ncn = 0;
        if (r0 + nv < M) {
          round_range(__builtin_amdgcn_readlane(e, nv - 1u), A, Z, IBn, ncn);
          pf_IB = IBn;
        } else if (next_task < t_hi) {
          const uint32_t An = __builtin_amdgcn_readfirstlane(na_l);
          const uint32_t Zn = __builtin_amdgcn_readlane(
              nb_l, min(n - next_task * TASK_STR, (uint32_t)TASK_STR) - 1u);
          round_range(An, An, Zn, IBn, ncn);
          pf_IB = IBn;
        }
        if (pf_IB != 0xFFFFFFFFu) {
          const uint4 *gn = reinterpret_cast<const uint4 *>(src + IBn);
#pragma unroll
          for (uint32_t u = 0; u < kPF; ++u)
            if (lane + WAVE * u < ncn) pf[u] = dd_ld16(gn + lane + WAVE * u);
        }
        pf_n = ncn;
      }
      WSTAMP(1);
      if (carry_exit < DD_NONE) carry_exit -= 8u * (IB - IB_prev);
      IB_prev = IB;
      const uint32_t bs = 8u * (s - IBX);
      const uint32_t bend = 8u * (min(b, e + 8u) - IBX);
      const uint32_t bstop = last ? bend : 8u * (e - IBX);
      DISink sk(my_ob);
      // ---- warm-up of the later items: to the first boundary >= 8 s
      uint32_t entry = bs;
      bool dead = false;  // EOS during the warm-up: entry unknown (re-decoded)
      constexpr bool kWMerge = DD_WMERGE && DD_MERGE && BI == 0;
      if (spec && !kWMerge) {  // (kWMerge: the first pass of the verify loop)
        uint32_t bp = 8u * (s - DD_OV - IBX);
        DiscardSink dk;
        const DDRun rw = dd_run<DiscardSink, DD_WSYNC != 0>(S.T, inp, bp, bs, bend, dk, dctr DD_SPASS);
        entry = bp;
        dead = rw.failed;
      }
      WSTAMP(2);
      // ---- the item's symbols
      uint32_t bp = entry;
      DDRun rr;
      rr.failed = rr.at_end = false;
      rr.t = rr.win = 0;
      // (DD_CKPT) a codeword boundary on the speculative path of a later
      // item, DD_CKB bits or so past its entry, and the symbols before it
      uint32_t cp_pos = XUNKNOWN, cp_cnt = 0;
      constexpr bool kMerge = DD_MERGE && BI == 0;
      if (valid && !dead && !kMerge) {  // (kMerge: in the verify loop's first pass)
        if (DD_CKPT && spec) {
          // the fast pairs up to the checkpoint, then the rest of the item
          const DDRun ra = dd_run<DISink, false, true>(S.T, inp, bp, bstop, bend, sk,
                                                       dctr DD_SPASS, (int32_t)(entry + DD_CKB));
          if (ra.failed) {
            rr.failed = true;  // EOS before the checkpoint
          } else {
            cp_pos = bp;
            cp_cnt = sk.count();
            rr = dd_run(S.T, inp, bp, bstop, bend, sk, dctr DD_SPASS);
          }
        } else {
          rr = dd_run(S.T, inp, bp, bstop, bend, sk, dctr DD_SPASS);
        }
      }
      uint32_t my_exit = rr.failed ? XFAIL : bp;
      uint32_t my_entry = dead ? XUNKNOWN : entry;
      uint32_t c0 = sk.count();
      WSTAMP(3);
      // ---- verify the later items against the previous item's exit
      // (DD_MERGE: one inlined decoder for the item and its re-decodes -- a
      // pass decodes the lanes marked run_ from `start`, then verifies)
      // (kWMerge: the warm-up is that decoder's first pass too, to the first
      // boundary >= bs through its careful steps, its symbols written and
      // then overwritten; a tail or EOS before bs leaves the entry unknown)
      bool run_ = kWMerge ? spec : (kMerge && valid && !dead);
      bool warm = kWMerge;  // (uniform) this pass is the warm-up
      uint32_t start = kWMerge ? 8u * (s - DD_OV - IBX) : entry;
      for (uint32_t iter = 0; iter <= WAVE + (kWMerge ? 2u : kMerge ? 1u : 0u); ++iter) {
        if (kMerge && __ballot(run_)) {
          if (run_) {
            DISink s3(my_ob);
            uint32_t bq = start;
            const DDRun r2 = dd_run(S.T, inp, bq, warm ? bs : bstop, bend, s3, dctr DD_SPASS);
            if (warm) {
              entry = bq;
              dead = r2.failed || bq < bs;
            } else {
              rr = r2;
              my_exit = rr.failed ? XFAIL : bq;
              c0 = s3.count();
            }
          }
          run_ = false;
        }
        if (kWMerge && warm) {  // the item pass next
          warm = false;
          my_entry = dead ? XUNKNOWN : entry;
          my_exit = entry;
          start = entry;
          run_ = valid && !dead;
          continue;
        }
        const uint32_t up = __shfl_up(my_exit, 1, 64);
        const uint32_t pred = lane ? up : carry_exit;
        const bool mism = spec && (my_entry != pred || my_entry == XUNKNOWN);
        const uint64_t bal = __ballot(mism);
        if (bal == 0) break;
        DCTR(3);
        const bool pred_mism = lane && ((bal >> (lane - 1u)) & 1u);
        if (mism && !pred_mism) {
          DISink s3(my_ob);
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
            bool fixed = false;
            if (DD_CKPT && cp_pos != XUNKNOWN && pred <= cp_pos) {
              // the true path from pred usually meets the speculative one
              // within a few symbols: if it reaches the checkpoint, the
              // symbols from there on are right already -- count the true
              // symbols before it, move the rest to follow them, write them
              uint32_t bq = pred;
              NullSink ns;
              const DDRun rc = dd_run(S.T, inp, bq, cp_pos, bend, ns, dctr DD_SPASS);
              if (!rc.failed && bq == cp_pos) {
                const uint32_t m = ns.count(), L = c0 - cp_cnt;
                lds_u8 *o = my_ob;
                if (m > cp_cnt) {
                  for (uint32_t j = L; j-- > 0;) o[m + j] = o[cp_cnt + j];
                } else if (m < cp_cnt) {
                  for (uint32_t j = 0; j < L; ++j) o[m + j] = o[cp_cnt + j];
                }
                // (a sink may write up to two bytes past its count)
                const uint8_t k0 = o[m], k1 = o[m + 1u];
                uint32_t bq2 = pred;
                DISink s4(my_ob);
                dd_run(S.T, inp, bq2, cp_pos, bend, s4, dctr DD_SPASS);
                if (L > 0u) o[m] = k0;
                if (L > 1u) o[m + 1u] = k1;
                c0 = m + L;
                fixed = true;  // (exit and tail: the speculative path's)
              }
            }
            if (!fixed) {
              uint32_t bq = pred;
              rr = dd_run(S.T, inp, bq, bstop, bend, s3, dctr DD_SPASS);
              my_exit = rr.failed ? XFAIL : bq;
              c0 = s3.count();
            }
          }
          my_entry = pred;
        }
      }
      WSTAMP(4);
      // ---- string symbol counts: segmented scan (heads: first items)
      // (the plain inclusive scan of the lanes' byte counts, less its value
      // before the lane's last head; no head yet: plus the carried count)
      const uint32_t V = valid ? c0 : 0u;
      const uint32_t Tinc = wave_incl_scan(V);
      const uint32_t h1 = wave_incl_max((!valid || k == 0) ? lane + 1u : 0u);
      const uint32_t excl_h = __shfl(Tinc - V, h1 ? h1 - 1u : 0u, 64);
      const uint32_t seg = h1 ? Tinc - excl_h : Tinc + carry_cnt;  // inclusive
      if (kLate) {  // the staging buffer is free: the next round's input into it
        staged_IB = pf_IB;
        if (pf_IB != 0xFFFFFFFFu) stage_pf(pf_n);
        // every load of the wave has landed (the offsets two tasks ahead
        // included): said explicitly, so no wait for them is placed after
        // this round's stores (vmcnt(0): expcnt and lgkmcnt left at max)
        __builtin_amdgcn_s_waitcnt(0x0F70);
      }
      if (valid && last)
        dd_finish(S.T, rr.failed, rr.t, rr.win, seg,
                  task_ovf && auto_slot(b - off0, t0 + i + 1u) > dst_cap, t0 + i, status,
                  fstate_out, flags_out);
      // ---- dense placement
      const uint32_t O_l = run + Tinc - V;
      if (valid && k == 0) ost[i] = O_l;
      WSTAMP(5);
      if (!DD_ABL_NOSTORE && DD_CSTORE && (IP >= 64u || DD_CSTORE == 2)) {
        // The round's bytes are the task's output [R0g, R1g): each lane moves
        // its region into the round's global dwords [W0, W1), laid out back
        // to back over the regions (realigned by alignbyte; the words shared
        // by two lanes OR'ed), then the wave stores them 16 bytes per lane.
        // The partial last word is carried into the next round (the task's
        // last one is written whole: the next task starts 4-aligned).
        const uint32_t Tot = __builtin_amdgcn_readlane(Tinc, 63);
        const uint64_t R0g = tbase + run, R1g = R0g + Tot, W0 = R0g >> 2;
        const uint64_t g0 = tbase + O_l;
        const uint32_t h = (uint32_t)((4u - (g0 & 3u)) & 3u);  // bytes before alignment
        const uint32_t nfull = V >= h ? (V - h) >> 2 : 0u;      // whole dwords
        const uint32_t mx = __builtin_amdgcn_readlane(wave_incl_max(nfull), 63);
        const uint32_t d0 = my_ob32[0];
        const uint32_t vt = __builtin_amdgcn_alignbyte(my_ob32[nfull + 1u], my_ob32[nfull], h);
        uint32_t d[di_rb(IP) / 4 + 1];
#pragma unroll
        for (uint32_t m0 = 0; m0 <= di_rb(IP) / 4; m0 += 4) {
          if (m0 > mx) break;
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j)
            if (m0 + j <= di_rb(IP) / 4) d[m0 + j] = my_ob32[m0 + j];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        lds_u32 *D = (lds_u32 *)S.ob[wv];
        const uint32_t nwr = (uint32_t)(((R1g + 3u) >> 2) - W0);  // the round's words
        for (uint32_t i = lane; i < nwr; i += WAVE) D[i] = 0u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane == 0 && ocarry) atomicOr((uint32_t *)&D[0], ocarry);
        if (V) {
          const uint32_t wb = (uint32_t)((g0 >> 2) - W0);
          if (h) {  // my first bytes share a word with the lanes before
            const uint32_t nh = min(h, V);
            const uint32_t mk = (nh == 4u ? 0xFFFFFFFFu : (1u << (8u * nh)) - 1u) << (8u * (4u - h));
            atomicOr((uint32_t *)&D[wb], (d0 << (8u * (4u - h))) & mk);
          }
          const uint32_t wf = wb + (h ? 1u : 0u);
#pragma unroll
          for (uint32_t m0 = 0; m0 < di_rb(IP) / 4; m0 += 4) {
            if (m0 >= mx) break;
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
              const uint32_t m = m0 + j;
              if (m < di_rb(IP) / 4 && m < nfull) D[wf + m] = __builtin_amdgcn_alignbyte(d[m + 1u], d[m], h);
            }
          }
          const uint32_t xt = h + 4u * nfull;
          if (V > xt) atomicOr((uint32_t *)&D[wf + nfull], vt & ((1u << (8u * (V - xt))) - 1u));
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const bool lastr = r0 + nv >= M;
        const uint32_t nst = lastr ? nwr : (uint32_t)((R1g >> 2) - W0);
        for (uint32_t i4 = 4u * lane; i4 < nst; i4 += 4u * WAVE) {
          const uint64_t gq = 4ull * (W0 + i4);
          if (i4 + 4u <= nst && gq + 16u <= dst_cap) {
            const u32x4 v = *(const lds_u32x4 *)(D + i4);
            *reinterpret_cast<uint4 *>(dst + gq) = make_uint4(v.x, v.y, v.z, v.w);
          } else {
            for (uint32_t u = 0; u < 4u && i4 + u < nst; ++u) {
              const uint32_t v = D[i4 + u];
              const uint64_t q = gq + 4u * u;
              if (q + 4u <= dst_cap) {
                *reinterpret_cast<uint32_t *>(dst + q) = v;
              } else {
                for (uint32_t y = 0; y < 4u; ++y)
                  if (q + y < dst_cap) dst[q + y] = (uint8_t)(v >> (8u * y));
              }
            }
          }
        }
        ocarry = (!lastr && nst < nwr) ? __builtin_amdgcn_readfirstlane(D[nst]) : 0u;
      } else if (!DD_ABL_NOSTORE) {
        // dwords realigned to the output (alignbyte) for as many dwords as
        // the wave's longest region, four per step; the bytes before the
        // first aligned dword and after the last one stored singly
        const uint64_t g0 = tbase + O_l;
        const uint32_t h = (uint32_t)((4u - (g0 & 3u)) & 3u);  // bytes before alignment
        const bool fits = g0 + V <= dst_cap;
        const uint32_t nfull = V >= h ? (V - h) >> 2 : 0u;      // whole dwords
        const uint32_t mx = __builtin_amdgcn_readlane(wave_incl_max(fits ? nfull : 0u), 63);
        uint32_t prev = my_ob32[0];
        const uint32_t d0 = prev;
#pragma unroll
        for (uint32_t m0 = 0; m0 < di_rb(IP) / 4; m0 += 4) {
          if (m0 >= mx) break;
          uint32_t c[4];
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j) c[j] = m0 + j < di_rb(IP) / 4 ? my_ob32[m0 + j + 1u] : 0u;
          uint32_t v[4];
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j) v[j] = __builtin_amdgcn_alignbyte(c[j], j ? c[j - 1] : prev, h);
          if (DD_ST4 && m0 + 4u <= nfull && fits) {
            // four whole dwords as one (dword-aligned) 16-byte store
            dd_st16(reinterpret_cast<uint4 *>(dst + g0 + h + 4u * m0), make_uint4(v[0], v[1], v[2], v[3]));
          } else {
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
              if (m0 + j < nfull && fits) *reinterpret_cast<uint32_t *>(dst + g0 + h + 4u * (m0 + j)) = v[j];
          }
          prev = c[3];
        }
        if (V) {
          const uint32_t vt = __builtin_amdgcn_alignbyte(my_ob32[nfull + 1u], my_ob32[nfull], h);
          const uint32_t nh = min(h, V);
          const uint32_t xt = h + 4u * nfull, ntl = V > xt ? V - xt : 0u;
          if (DD_HT2 && fits) {
            // the head up to alignment and the tail after the last whole
            // dword as (aligned) 2-byte stores plus at most one byte each
            if (nh == h) {
              if (h & 1u) dst[g0] = (uint8_t)d0;
              if (h & 2u) *reinterpret_cast<uint16_t *>(dst + g0 + (h & 1u)) = (uint16_t)(d0 >> (8u * (h & 1u)));
            } else {
              for (uint32_t x = 0; x < nh; ++x) dst[g0 + x] = (uint8_t)(d0 >> (8u * x));
            }
            if (ntl & 2u) *reinterpret_cast<uint16_t *>(dst + g0 + xt) = (uint16_t)vt;
            if (ntl & 1u) dst[g0 + xt + (ntl & 2u)] = (uint8_t)(vt >> (8u * (ntl & 2u)));
          } else {
#pragma unroll
            for (uint32_t x = 0; x < 3u; ++x) {
              if (x < nh && fits) dst[g0 + x] = (uint8_t)(d0 >> (8u * x));
              if (x < ntl && fits) dst[g0 + xt + x] = (uint8_t)(vt >> (8u * x));
            }
          }
          if (!fits) {  // near dst_cap: byte by byte, nothing at or past it
            for (uint32_t x = 0; x < V; ++x)
              if (g0 + x < dst_cap) dst[g0 + x] = my_ob[x];
          }
        }
      }
      WSTAMP(6);
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
      dst_off[t0 + lane] = (uint32_t)min(tbase + ost[lane], dst_cap);
      if (t0 + lane == n - 1u) dst_off[n] = (uint32_t)min(tbase + run, dst_cap);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    task = next_task;
    if (kLate) rotate();
  }
  WSTAMP_FLUSH_W(IW);
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
// HPACK string literals: emit_string (lib/nghttp2_hd.c:1001-1044), batched
// ---------------------------------------------------------------------------
// A literal is the H bit (0x80 iff the Huffman form is strictly shorter,
// :1011) with the payload length as a 7-bit-prefix integer
// (count_encoded_length / encode_length, :823-863), then the payload: the
// Huffman bytes or the raw ones.  After a batch encode into the workspace,
// k_frame_len sizes each literal, a tile scan places them, and k_frame_copy
// writes the output stream dword by dword (coalesced stores), gathering each
// byte from the prefix, the Huffman pool or the raw pool.

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

// out_len[s] = literal bytes of string s; tile sums for the offset scan.
__global__ __launch_bounds__(WG) void k_frame_len(const uint32_t *__restrict__ src_off,
                                                  const uint32_t *__restrict__ enc_off, uint32_t n,
                                                  uint32_t *__restrict__ out_len,
                                                  uint32_t *__restrict__ tile_sums) {
  __shared__ uint32_t red[WG / 64];
  const uint32_t s = blockIdx.x * WG + threadIdx.x;
  uint32_t f = 0;
  if (s < n) {
    const uint32_t R = src_off[s + 1] - src_off[s], E = enc_off[s + 1] - enc_off[s];
    const uint32_t P = E < R ? E : R;
    f = prefix7_len(P) + P;
    out_len[s] = f;
  }
  uint32_t tot;
  block_excl_scan<WG>(f, red, &tot);
  if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
}

// One workgroup per tile of 256 literals: the tile's output bytes
// [dst_off[t0], dst_off[t0 + 256]) go out as dwords, one per thread and
// pass; a dword shared with a neighbouring tile goes bytewise.
__global__ __launch_bounds__(WG) void k_frame_copy(const uint8_t *__restrict__ src,
                                                   const uint32_t *__restrict__ src_off,
                                                   const uint8_t *__restrict__ enc,
                                                   const uint32_t *__restrict__ enc_off, uint32_t n,
                                                   uint8_t *__restrict__ dst, uint64_t dst_cap,
                                                   const uint32_t *__restrict__ dst_off) {
  __shared__ uint32_t fo[WG + 1];   // literal starts (tile-relative to nothing: absolute)
  __shared__ uint32_t pay[WG];      // payload length | H << 31
  __shared__ uint32_t psrc[WG];     // payload source offset (enc or src pool)
  __shared__ uint8_t plen[WG];
  const uint32_t t0 = blockIdx.x * WG;
  const uint32_t nt = min(n - t0, (uint32_t)WG);
  const uint32_t s = t0 + threadIdx.x;
  if (threadIdx.x < nt) {
    const uint32_t a = src_off[s], R = src_off[s + 1] - a;
    const uint32_t e = enc_off[s], E = enc_off[s + 1] - e;
    const bool h = E < R;
    const uint32_t P = h ? E : R;
    fo[threadIdx.x] = dst_off[s];
    pay[threadIdx.x] = P | (h ? 0x80000000u : 0u);
    psrc[threadIdx.x] = h ? e : a;
    plen[threadIdx.x] = (uint8_t)prefix7_len(P);
  }
  if (threadIdx.x == 0) fo[nt] = dst_off[t0 + nt];
  __syncthreads();
  const uint32_t lo = fo[0], hi = fo[nt];
  if (hi == lo) return;
  for (uint32_t w = (lo >> 2) + threadIdx.x; w <= ((hi - 1u) >> 2); w += WG) {
    const uint32_t p0 = 4u * w;
    // the literal holding the first in-range byte of this dword
    const uint32_t pf = max(p0, lo);
    uint32_t a = 0, b = nt - 1u;
    while (a < b) {  // last i with fo[i] <= pf
      const uint32_t m = (a + b + 1u) >> 1;
      if (fo[m] <= pf) a = m; else b = m - 1u;
    }
    uint32_t i = a, v = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4u; ++j) {
      const uint32_t p = p0 + j;
      if (p < lo || p >= hi) continue;
      while (p >= fo[i + 1]) ++i;  // empty literals do not exist: each has >= 1 byte
      const uint32_t r = p - fo[i], L = plen[i], P = pay[i] & 0x7FFFFFFFu;
      const bool h = pay[i] >> 31;
      uint32_t byte;
      if (r < L) byte = prefix7_byte(P, h ? 1u : 0u, r);
      else byte = (h ? enc : src)[psrc[i] + (r - L)];
      v |= byte << (8u * j);
    }
    if (p0 >= lo && p0 + 4u <= hi && p0 + 4u <= dst_cap) {
      *reinterpret_cast<uint32_t *>(dst + p0) = v;
    } else {
      for (uint32_t j = 0; j < 4u; ++j) {
        const uint32_t p = p0 + j;
        if (p >= lo && p < hi && p < dst_cap) dst[p] = (uint8_t)(v >> (8u * j));
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Lane decoder (DESIGN.md "decode"): one lane decodes one whole string
// (lib/nghttp2_hd_huffman.c:111-143 with fin = 1, exact entries -- no pieces,
// no warm-up, no verify).
//
// A workgroup owns a contiguous window of strings and orders it by encoded
// length in LDS (128 length classes, longest first); its waves then claim
// groups of 64 strings of that order, one string per lane, so the lanes of
// a wave have about the same number of bits to decode and the longest
// strings start first.  A lane's input streams through a 64-byte ring in LDS
// (four 16-byte chunks, dword-major so that the refill reads of the 64 lanes
// never share a bank); chunks are loaded DL_D periods before they are
// written to the ring, one (unconditional) load per period, so the wait for
// a chunk is a counted vmcnt that long loads have met.  The output goes
// through a 32-byte LDS buffer that leaves as whole 16-byte blocks.  Slots:
// decode_batch_auto's 16-byte aligned slots (dl_slot), or the caller's
// (decode_batch: only decoded bytes inside the slot are written).
// ---------------------------------------------------------------------------
#ifndef DL_WAVES
#define DL_WAVES 16
#endif
#ifndef DL_LB
#define DL_LB 13
#endif
#ifndef DL_D
#define DL_D 4         // staged chunk loads in flight per lane (periods of lead)
#endif
#ifndef DL_STAMPS
#define DL_STAMPS 0    // diagnostic build only: per-wave phase cycles
#endif
#ifndef DL_ABL
#define DL_ABL 0       // ablation builds only (tools/diag): 1 no fast-period stores, 2 no staged loads
#endif
#ifndef DL_LDP
#define DL_LDP 0       // cache policy of the staged chunk loads (A/B builds: 1 nt, 2 sc0 sc1)
#endif
#ifndef DL_STP
#define DL_STP 0       // cache policy of the block stores (A/B builds: 1 nt)
#endif
#if DL_LDP == 1
#define DL_LDPOL " nt"
#elif DL_LDP == 2
#define DL_LDPOL " sc0 sc1"
#else
#define DL_LDPOL ""
#endif
#if DL_STP == 1
#define DL_STPOL " nt"
#else
#define DL_STPOL ""
#endif
#define DL_NT (WAVE * DL_WAVES)
#define DL_P 3u        // pairs per period (one input / output service per period)
#define DL_RING 16u    // input ring dwords per lane (four chunks)
#define DL_OB 32u      // output buffer bytes per lane
#define DL_CLASSES 128u
#define DL_WMAX 8192u  // strings sorted at once by a workgroup
#define DL_NONE 0xFFFFFFFFu
#define DL_OOB 0xFFFFFFF0u  // a buffer offset past every descriptor's range

struct DLShared {
  DecT<DL_LB> T;                                        // the lookup at LDS offset 0
  uint32_t ring[DL_WAVES][DL_RING * WAVE];              // dword j of lane l at [64 j + l]
  uint32_t ob[DL_WAVES][DL_OB / 4 * WAVE];             // output dword j of lane l at [64 j + l]
  uint16_t order[DL_WMAX];                              // the window in decode order
  uint32_t hist[DL_CLASSES];
  uint32_t claimed;
};

#if DL_STAMPS
__device__ unsigned long long g_dl_stamps[2048][12];
#define DLS_INIT() unsigned long long dls[12] = {}, dlt = __builtin_amdgcn_s_memtime(), dlb = dlt
#define DLS(slot)                                                              \
  do {                                                                         \
    const unsigned long long t1_ = __builtin_amdgcn_s_memtime();               \
    dls[slot] += t1_ - dlt;                                                    \
    dlt = t1_;                                                                 \
  } while (0)
#define DLS_CNT(slot) (++dls[slot])
#define DLS_FLUSH()                                                            \
  do {                                                                         \
    dls[11] = __builtin_amdgcn_s_memtime() - dlb;                              \
    if (lane == 0)                                                             \
      for (int s_ = 0; s_ < 12; ++s_) g_dl_stamps[(blockIdx.x * DL_WAVES + wv) & 2047][s_] = dls[s_]; \
  } while (0)
#else
#define DLS_INIT() do { } while (0)
#define DLS(slot) do { } while (0)
#define DLS_CNT(slot) do { } while (0)
#define DLS_FLUSH() do { } while (0)
#endif

// (an explicit integer minimum: HIP's min() picks a floating overload for
// 64-bit integers)
__device__ __host__ __forceinline__ uint64_t u64min(uint64_t a, uint64_t b) { return a < b ? a : b; }

// decode_batch_auto's slot of string s: 16 * (ceil(floor(8 x_s / 5) / 16) + s),
// x_s = off[s] - off[0].  Each slot is 16-byte aligned and a multiple of 16
// bytes, at least floor(8 E_s / 5) + 1 (the reference's allocation,
// lib/nghttp2_hd.c:2080-2082), so whole 16-byte blocks of a string's output
// stay inside its slot.
__device__ __host__ __forceinline__ uint64_t dl_slot(uint32_t x, uint32_t s) {
  const uint64_t g = ((uint64_t)x * 8u) / 5u;
  return 16u * (((g + 15u) >> 4) + s);
}

// Length class, 0 = longest: 2-byte classes below 64 encoded bytes, 8 up to
// 256, 32 up to 1 KiB, 128 up to 4 KiB, then powers of two.
__device__ __forceinline__ uint32_t dl_class(uint32_t E) {
  uint32_t c;
  if (E < 64u) c = E >> 1;
  else if (E < 256u) c = 32u + ((E - 64u) >> 3);
  else if (E < 1024u) c = 56u + ((E - 256u) >> 5);
  else if (E < 4096u) c = 80u + ((E - 1024u) >> 7);
  else c = min(104u + (31u - (uint32_t)__builtin_clz(E)) - 12u, DL_CLASSES - 1u);
  return DL_CLASSES - 1u - c;
}

// Chunk staging in AGPRs (this kernel has no MFMA; nothing else of the
// compiler's lives there): slot J is a[4J .. 4J+3], written only by these
// inline-asm loads and read only after an explicit counted wait, so no load
// is ever in flight into a register the compiler owns (cdna_hip_programming.md
// 5.7 item 1; nghttp2_amd/tools/check_agpr.py audits every build).  The
// compiler does not count these loads: its own waits are not pulled down to
// them.  The fast periods' loads and stores are exec-masked to the lanes that
// have a chunk to take or a block to store (out-of-range lanes would still
// take address-unit cycles), and each is issued every period -- with one lane
// at an out-of-range offset when no lane has one, so EXEC is never 0 -- so
// that every period issues exactly one load and one store.
#define DL_AG_LOAD(A0, A1, A2, A3, AR)                                                   \
  asm volatile("v_cmp_ne_u32 vcc, 0, %1\n\ts_nop 1\n\ts_and_saveexec_b64 %0, vcc\n\t"   \
               "s_nop 4\n\tbuffer_load_dwordx4 " AR ", %2, %3, 0 offen" DL_LDPOL "\n\t"   \
               "s_mov_b64 exec, %0"                                                      \
               : "=&s"(saved)                                                            \
               : "v"(pred), "v"(voff), "s"(rsrc)                                         \
               : "vcc", A0, A1, A2, A3, "memory")
template <int J>
__device__ __forceinline__ void dl_stage_load(uint32_t pred, uint32_t voff, __amdgpu_buffer_rsrc_t rsrc) {
  uint64_t saved;
  if (J == 0) DL_AG_LOAD("a0", "a1", "a2", "a3", "a[0:3]");
  if (J == 1) DL_AG_LOAD("a4", "a5", "a6", "a7", "a[4:7]");
  if (J == 2) DL_AG_LOAD("a8", "a9", "a10", "a11", "a[8:11]");
  if (J == 3) DL_AG_LOAD("a12", "a13", "a14", "a15", "a[12:15]");
}
#undef DL_AG_LOAD
// a 16-byte store by the lanes with pred set (same issue rule); the trailing
// s_nop keeps the next instruction off the data registers until the store
// has read them
__device__ __forceinline__ void dl_store16(uint32_t pred, uint32_t voff, u32x4 data,
                                           __amdgpu_buffer_rsrc_t rsrc) {
  uint64_t saved;
  asm volatile("v_cmp_ne_u32 vcc, 0, %1\n\ts_nop 1\n\ts_and_saveexec_b64 %0, vcc\n\t"
               "s_nop 4\n\tbuffer_store_dwordx4 %3, %2, %4, 0 offen" DL_STPOL "\n\ts_mov_b64 exec, %0\n\ts_nop 1"
               : "=&s"(saved)
               : "v"(pred), "v"(voff), "v"(data), "s"(rsrc)
               : "vcc", "memory");
}
// The staged chunk of slot J, after its load: N younger memory instructions
// may still be in flight (every fast period issues one load and one store, so
// the load of DL_D periods ago has 2 DL_D - 1 younger ones).
#define DL_AG_READ(N, A0, A1, A2, A3)                                                    \
  asm volatile("s_waitcnt vmcnt(" #N ")\n\tv_accvgpr_read_b32 %0, " A0                   \
               "\n\tv_accvgpr_read_b32 %1, " A1 "\n\tv_accvgpr_read_b32 %2, " A2         \
               "\n\tv_accvgpr_read_b32 %3, " A3                                          \
               : "=v"(v.x), "=v"(v.y), "=v"(v.z), "=v"(v.w)                              \
               :                                                                         \
               : "memory")
template <int J>
__device__ __forceinline__ u32x4 dl_stage_read() {
  u32x4 v;
  if (J == 0) DL_AG_READ(7, "a0", "a1", "a2", "a3");
  if (J == 1) DL_AG_READ(7, "a4", "a5", "a6", "a7");
  if (J == 2) DL_AG_READ(7, "a8", "a9", "a10", "a11");
  if (J == 3) DL_AG_READ(7, "a12", "a13", "a14", "a15");
  return v;
}
#undef DL_AG_READ
__device__ __forceinline__ void dl_stage_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

template <bool AUTO>
__global__ __launch_bounds__(DL_NT) void k_decode_lanes(const uint8_t *__restrict__ src,
                                                        const uint32_t *__restrict__ off, uint32_t n,
                                                        uint32_t win, uint32_t sorted,
                                                        uint8_t *__restrict__ dst, uint64_t dst_cap,
                                                        uint32_t *__restrict__ dst_off,
                                                        int32_t *__restrict__ status,
                                                        uint16_t *__restrict__ fstate_out,
                                                        uint8_t *__restrict__ flags_out) {
  __shared__ DLShared S;
  constexpr uint32_t LB = DL_LB, G2 = 2u * DL_LB;  // a fast pair needs 2 LB bits of the string
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  lds_u32 *ring = (lds_u32 *)S.ring[wv] + lane;
  lds_u32 *ob = (lds_u32 *)S.ob[wv] + lane;
  stage_dec_tables(S.T, DL_NT);
  const DecT<DL_LB> &T = S.T;
  DLS_INIT();
  const uint32_t off0 = __builtin_amdgcn_readfirstlane(off[0]);
  // buffer descriptors: reads past the pool's readable end (align16(off[n]) +
  // 16) and stores past dst_cap are dropped, so a lane with nothing to load or
  // store in a period issues its load / store at DL_OOB
  const uint32_t src_lim = __builtin_amdgcn_readfirstlane(
      (uint32_t)u64min((((uint64_t)off[n] + 15u) & ~15ull) + 16u, (uint64_t)DL_OOB));
  // (inputs made provably uniform, so the compiler keeps the descriptors in
  // SGPRs instead of wrapping every buffer op in a waterfall loop)
  auto uni_ptr = [](const void *p) -> void * {
    const uint64_t v = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (void *)(uintptr_t)(((uint64_t)hi << 32) | lo);
  };
  void *const src_u = uni_ptr(src);
#define DL_RD() __builtin_amdgcn_make_buffer_rsrc(src_u, 0, (int)src_lim, 0x00020000)
  const uint32_t dst_lim = __builtin_amdgcn_readfirstlane((uint32_t)(AUTO ? u64min(dst_cap, (uint64_t)DL_OOB) : DL_OOB));
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(uni_ptr(dst), 0, (int)dst_lim, 0x00020000);
  // this workgroup's window of strings, sorted DL_WMAX at a time
  const uint32_t r0 = min(n, blockIdx.x * win), r1 = min(n, r0 + win);
  for (uint32_t w0 = r0; w0 < r1; w0 += DL_WMAX) {
    const uint32_t wn = min(DL_WMAX, r1 - w0), ngr = (wn + 63u) / 64u;
    __syncthreads();  // (the previous sub-window's waves are done with order[])
    if (sorted) {
      for (uint32_t c = threadIdx.x; c < DL_CLASSES; c += DL_NT) S.hist[c] = 0u;
      __syncthreads();
      constexpr uint32_t PT = DL_WMAX / DL_NT;
      uint32_t cls[PT];
#pragma unroll
      for (uint32_t u = 0; u < PT; ++u) {
        const uint32_t t = threadIdx.x + u * DL_NT;
        cls[u] = t < wn ? dl_class(off[w0 + t + 1] - off[w0 + t]) : 0u;
        if (t < wn) atomicAdd((uint32_t *)&S.hist[cls[u]], 1u);
      }
      __syncthreads();
      if (wv == 0) {  // exclusive scan of the 128 class counts, two per lane
        const uint32_t h0 = S.hist[2u * lane], h1 = S.hist[2u * lane + 1u];
        const uint32_t inc = wave_incl_scan(h0 + h1);
        S.hist[2u * lane] = inc - h0 - h1;
        S.hist[2u * lane + 1u] = inc - h1;
      }
      __syncthreads();
#pragma unroll
      for (uint32_t u = 0; u < PT; ++u) {
        const uint32_t t = threadIdx.x + u * DL_NT;
        if (t < wn) S.order[atomicAdd((uint32_t *)&S.hist[cls[u]], 1u)] = (uint16_t)t;
      }
    }
    if (threadIdx.x == 0) S.claimed = 0u;
    __syncthreads();
    DLS(0);
    // Groups are claimed one ahead: the next group's string offsets are
    // loaded when the current one starts, its first four input chunks when
    // the current one's fast phase ends.
    auto claim = [&]() -> uint32_t {
      uint32_t gi = 0;
      if (lane == 0) gi = atomicAdd((uint32_t *)&S.claimed, 1u);
      return __builtin_amdgcn_readfirstlane(gi);
    };
    auto load_meta = [&](uint32_t gg) -> uint4 {  // {string, first byte, end}
      const uint32_t q = gg * 64u + lane;
      if (gg >= ngr || q >= wn) return make_uint4(DL_NONE, 0u, 0u, 0u);
      const uint32_t s = w0 + (sorted ? (uint32_t)S.order[q] : q);
      return make_uint4(s, off[s], off[s + 1], 0u);
    };
    auto chunk_ok = [&](const uint4 &m, uint32_t j) {  // chunk j of the string (its bytes + 7 after)
      return m.x != DL_NONE && m.z >= m.y && m.y >= off0 && j <= ((m.z + 7u - (m.y & ~15u)) >> 4);
    };
    u32x4 cn[4];
    auto load_chunks = [&](const uint4 &m) {
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) {
        cn[j] = u32x4{0u, 0u, 0u, 0u};
        if (chunk_ok(m, j)) cn[j] = __builtin_amdgcn_raw_buffer_load_b128(DL_RD(), (m.y & ~15u) + 16u * j, 0, 0);
      }
    };
    uint32_t g = claim();
    uint4 mn = load_meta(g);
    load_chunks(mn);
    while (g < ngr) {
      DLS_CNT(9);
      const uint4 mc = mn;
      const bool have = mc.x != DL_NONE;
      const uint32_t i = have ? mc.x : 0u, a = mc.y, b = mc.z;
      const bool bad = have && (b < a || a < off0 || b - a >= (1u << 28));
      const bool act = have && !bad;
      const uint32_t E = act ? b - a : 0u;
      // ---- input: chunks 0..3 into the ring, the bit buffer from the first byte
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) {
        ring[64u * (4u * j)] = __builtin_bswap32(cn[j].x);
        ring[64u * (4u * j + 1u)] = __builtin_bswap32(cn[j].y);
        ring[64u * (4u * j + 2u)] = __builtin_bswap32(cn[j].z);
        ring[64u * (4u * j + 3u)] = __builtin_bswap32(cn[j].w);
      }
      const uint32_t gn = claim();
      mn = load_meta(gn);
      // ---- output window [o, o + cap)
      uint32_t o = 0, cap = 0;
      bool slot_ovf = false;
      if (AUTO) {
        const uint64_t s0 = dl_slot(a - off0, i), s1 = act ? dl_slot(b - off0, i + 1u) : s0;
        o = (uint32_t)u64min(s0, dst_cap);
        cap = (uint32_t)(u64min(s1, dst_cap) - o);
        slot_ovf = s1 > dst_cap;
        if (have) {
          dst_off[i] = o;
          if (i == n - 1u) dst_off[n] = (uint32_t)u64min(dl_slot(off[n] - off0, n), dst_cap);
        }
      } else if (have) {
        o = dst_off[i];
        const uint32_t o1 = dst_off[i + 1];
        cap = o1 >= o ? o1 - o : 0u;
      }
      const uint32_t c0 = a & ~15u;
      const uint32_t jmax = act ? (b + 7u - c0) >> 4 : 0u;  // the last chunk the lane reads
      const uint32_t m0 = (a & 15u) >> 2, r8 = 8u * (a & 3u);
      // bb: the stream bits from the string's first one, MSB first, nb of them
      // (the valid bits always end on a stream dword boundary)
      uint64_t bb = ((((uint64_t)ring[64u * m0]) << 32) | ring[64u * (m0 + 1u)]) << r8;
      uint32_t nb = 64u - r8, k = m0 + 2u;  // k: the next ring dword to take, prefetched in nxt
      uint32_t nxt = ring[64u * k];
      uint32_t rem = 8u * E;           // string bits left
      // chunk staging: slot j (visited every DL_D-th period) holds chunk sc[j]
      // until its visit commits it to the ring; a chunk is loaded only once
      // its ring rows are free, so that visit always commits it
      uint32_t cc = 4u, nl = 4u;       // chunks committed to the ring / the next one to load
      uint32_t sc[DL_D];
#pragma unroll
      for (uint32_t j = 0; j < DL_D; ++j) sc[j] = DL_NONE;
      // ---- output: the decoded bytes gather in a 64-bit register (acc, nacc
      // bits, little-endian) and leave it as whole dwords into the lane's
      // 8-dword LDS ring (dword q of the output from G0 = o & ~15 at row q & 7;
      // wq dwords complete, the partial one is rewritten in place at row wq).
      // Whole 16-byte blocks inside the window leave at once; a partial one
      // (the head of an unaligned caller slot, or the block across the
      // window's end) waits in registers for the string's end.
      const uint32_t G0 = o & ~15u;
      uint32_t G = G0, wq = (o & 15u) >> 2, fq = 0;  // fq: dwords flushed
      uint64_t acc = 0;
      uint32_t nacc = 8u * (o & 3u);
      const uint32_t wend = o + cap;
      u32x4 hv = {0, 0, 0, 0}, tv = {0, 0, 0, 0};
      uint32_t hG = DL_NONE, tG = DL_NONE;
      auto rdblk = [&]() {
        return u32x4{ob[64u * (fq & 7u)], ob[64u * ((fq + 1u) & 7u)], ob[64u * ((fq + 2u) & 7u)],
                     ob[64u * ((fq + 3u) & 7u)]};
      };
      auto flush = [&]() {  // exactly one store instruction per call (see dl_store16)
        const bool fl = wq - fq >= 4u;
        const u32x4 blk = rdblk();
        const bool full = fl && G >= o && G + 16u <= wend;
        const bool none = !__ballot(full);
        if (!(DL_ABL & 1)) dl_store16(full || (none && lane == 0u), full ? G : DL_OOB, blk, wr);
        if (fl) {
          if (!full && G < o) {
            hv = blk;
            hG = G;
          } else if (!full && G < wend && tG == DL_NONE) {
            tv = blk;
            tG = G;
          }
          fq += 4u;
          G += 16u;
        }
      };
// v: up to 4 output bytes (little-endian), bits = 8 x their count
#define DL_PUT(v, bits)                                                  \
  do {                                                                   \
    acc |= (uint64_t)(v) << nacc;                                        \
    nacc += (bits);                                                      \
    const bool em_ = nacc >= 32u;                                        \
    ob[64u * (wq & 7u)] = (uint32_t)acc;                                 \
    acc = em_ ? acc >> 32 : acc;                                         \
    nacc -= em_ ? 32u : 0u;                                              \
    wq += em_ ? 1u : 0u;                                                 \
  } while (0)
#define DL_REFILL()                                                      \
  do {                                                                   \
    const bool t_ = nb < 32u;                                            \
    bb |= (uint64_t)(t_ ? nxt : 0u) << ((32u - nb) & 63u);               \
    nb += t_ ? 32u : 0u;                                                 \
    k += t_ ? 1u : 0u;                                                   \
    nxt = ring[64u * (k & (DL_RING - 1u))];                              \
  } while (0)
      bool failed = false, stopf = false;  // stopf: the string's tail met in a fast pair
      DLS(1);
      // ---- fast periods: a service (store, commit, load), then DL_P pairs
      for (bool more = true; more;) {
        static_assert(DL_D == 4, "four AGPR staging slots, vmcnt(7)");
#pragma unroll
        for (uint32_t j = 0; j < DL_D; ++j) {
          const bool want = act && !failed && !stopf && rem >= G2;
          if (!__ballot(want)) {
            more = false;
            break;
          }
          DLS_CNT(10);
          flush();
          if (sc[j] != DL_NONE) {  // chunk cc, loaded DL_D periods ago
            u32x4 v = u32x4{0u, 0u, 0u, 0u};
            if (DL_ABL & 2) {
            } else if (j == 0) v = dl_stage_read<0>();
            else if (j == 1) v = dl_stage_read<1>();
            else if (j == 2) v = dl_stage_read<2>();
            else if (j == 3) v = dl_stage_read<3>();
            const uint32_t rr = 4u * (cc & 3u);
            ring[64u * rr] = __builtin_bswap32(v.x);
            ring[64u * (rr + 1u)] = __builtin_bswap32(v.y);
            ring[64u * (rr + 2u)] = __builtin_bswap32(v.z);
            ring[64u * (rr + 3u)] = __builtin_bswap32(v.w);
            ++cc;
            sc[j] = DL_NONE;
          }
          // one load per period (see dl_stage_load), by the lanes with a chunk
          // to take: the next one, once chunk nl - 4 is used up
          const bool ld = nl <= jmax && k >= 4u * (nl - 3u);
          const uint32_t lp = (ld || (!__ballot(ld) && lane == 0u)) ? 1u : 0u;
          const uint32_t voff = ld ? c0 + 16u * nl : DL_OOB;
          if (DL_ABL & 2) {
          } else if (j == 0) dl_stage_load<0>(lp, voff, DL_RD());
          else if (j == 1) dl_stage_load<1>(lp, voff, DL_RD());
          else if (j == 2) dl_stage_load<2>(lp, voff, DL_RD());
          else if (j == 3) dl_stage_load<3>(lp, voff, DL_RD());
          if (ld) sc[j] = nl++;
          DLS(2);
          // a lane runs its pairs when the ring holds the dwords they can
          // take (two per pair), or when every chunk of its string is in (the
          // ring rows past them are bits after the string end: never taken)
          bool run = want && (4u * cc - k >= 2u * DL_P + 1u || cc > jmax);
#pragma unroll
          for (uint32_t p = 0; p < DL_P; ++p) {
            if (run) {
              const uint32_t e1 = T.lut[(uint32_t)(bb >> 32) >> (32 - LB)];
              const uint32_t U1 = E_USED(e1);
              bb <<= U1;
              const uint32_t e2 = T.lut[(uint32_t)(bb >> 32) >> (32 - LB)];
              const uint32_t U2 = E_USED(e2);
              bb <<= U2;
              DL_PUT((e1 & 0xFFFFu) | ((e2 & 0xFFFFu) << E_CNT8(e1)), E_CNT8(e1) + E_CNT8(e2));
              nb -= U1 + U2;
              rem -= U1 + U2;
              DL_REFILL();
              if (e2 == 0u) {  // a code longer than the lookup (an e1 of 0 stalls e2 too)
                const uint32_t e_ = slow_entry(T, (uint32_t)(bb >> 32), rem);
                if (e_ == 0xFFFFFFFFu) {
                  failed = true;  // EOS: the FSM's sticky failure state
                } else if (E_L1(e_) > rem) {
                  stopf = true;   // the string's tail: the careful steps take it
                } else {
                  DL_PUT(e_ & 0xFFu, 8u);
                  const uint32_t U_ = E_USED(e_);
                  bb <<= U_;
                  nb -= U_;
                  rem -= U_;
                  DL_REFILL();
                }
              }
              run = !failed && !stopf && rem >= G2;
            }
          }
          DLS(3);
        }
      }
#undef DL_REFILL
      dl_stage_drain();  // (no staged load in flight past the fast periods)
      load_chunks(mn);  // the next group's first chunks, in flight over this one's tail
      flush();
      // ---- careful steps: the last < 2 LB bits (or a long code at the tail),
      // each step predicated on the string end instead of branching
      uint32_t t_bits = 0, t_win = 0;
      bool done = !act || failed;
      while (__ballot(!done)) {
        const uint32_t w = (uint32_t)(bb >> 32);
        const bool stop = done || rem == 0u;
        uint32_t e = T.lut[w >> (32 - LB)];
        const bool slow = e == 0u && !stop;
        if (__ballot(slow)) {
          if (slow) e = slow_entry(T, w, rem);
        }
        const bool eos = e == 0xFFFFFFFFu && !stop;
        const uint32_t L1 = E_L1(e), U = E_USED(e);
        const bool take1 = !stop && !eos && L1 <= rem;
        const bool take2 = take1 && E_CNT(e) == 2u && U <= rem;
        const bool tail = !stop && !eos && !take1;  // a proper prefix of a code
        t_bits = tail ? rem : t_bits;
        t_win = tail ? w : t_win;
        const uint32_t adv = take2 ? U : (take1 ? L1 : 0u);
        if (take1) DL_PUT(e & (take2 ? 0xFFFFu : 0xFFu), take2 ? 16u : 8u);
        bb <<= adv;
        rem -= adv;
        failed = failed || eos;
        done = done || eos || !take1 || rem == 0u;
      }
      DLS(4);
      ob[64u * (wq & 7u)] = (uint32_t)acc;  // the partial last dword
      // ---- the rest of the output, status and final decode context
      flush();
#undef DL_PUT
      const uint32_t nsym = G0 + 4u * wq + (nacc >> 3) - o;
      if (act) {
        // AUTO: the last block may hold bytes past the string (inside its slot)
        const uint32_t hi = AUTO ? wend : o + min(cap, nsym);
        auto put_bytes = [&](const u32x4 &v, uint32_t Gb) {
          for (uint32_t x = 0; x < 16u; ++x) {
            const uint32_t q = Gb + x;
            if (q >= o && q < hi) dst[q] = (uint8_t)(v[x >> 2] >> (8u * (x & 3u)));
          }
        };
        if (hG != DL_NONE) put_bytes(hv, hG);
        if (tG != DL_NONE) put_bytes(tv, tG);
        if (4u * wq + (nacc >> 3) > 4u * fq) {
          const u32x4 v = rdblk();
          if (G >= o && G + 16u <= hi) *reinterpret_cast<uint4 *>(dst + G) = make_uint4(v.x, v.y, v.z, v.w);
          else put_bytes(v, G);
        }
      }
      if (have) {
        if (bad) {
          status[i] = NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
          if (fstate_out) {
            fstate_out[i] = 0u;
            flags_out[i] = 0u;
          }
        } else {
          dd_finish(T, failed, t_bits, t_win, nsym, AUTO ? slot_ovf : nsym > cap, i, status,
                    fstate_out, flags_out);
        }
      }
      g = gn;
      DLS(5);
    }
  }
  DLS_FLUSH();
#undef DL_RD
}

// ---------------------------------------------------------------------------
// Lane decoder with cooperative transfers (DESIGN.md "decode"): one lane
// decodes one whole string, as k_decode_lanes, but no lane loads or stores
// its own bytes.  Global memory is touched only in whole 64-byte granules,
// 16 of them per instruction (lane 4q + c moves piece c of the q-th granule):
// a per-lane 16-byte access stream to a long string leaves partial lines in
// L2 that are evicted long before the lane's next piece arrives, so every
// piece cost a separate line fetch or a partial-line write.  Each period a
// wave ranks the lanes that wait for an input block (the next 64-byte
// aligned block of their string, once its ring rows are free) and the lanes
// holding a complete output block, pushes each one's {address | lane} to its
// loader quad (ds_permute + a quad broadcast), and issues at most L2_NI
// transfers each way.  Loaded blocks are committed to the owners' input rings
// in the next period; output blocks are read from the owners' rings, zeroed,
// and stored at once.
//
// Output slots are 64-byte aligned (dl2_slot), so a string's last block is
// stored whole (the bytes past the string inside its slot are zero): every
// store is a full granule.  Output bits are OR-ed into the lane's ring at
// the output bit position (ds_or, no read-modify-write in registers).
// ---------------------------------------------------------------------------
#ifndef L2_WAVES
#define L2_WAVES 10
#endif
#define L2_NT (WAVE * L2_WAVES)
#define L2_P 3u        // pairs per period
// Input ring: a 64-byte block plus L2_IN - 16 dwords of margin; block j is
// requested once dword 16 j - (L2_IN - 16) is taken, so a lane that runs a
// period (which needs 2 L2_P dwords at most) rarely waits for one.
#define L2_IN 24u
// Output ring: a period adds at most 5 L2_P bytes, so with every complete
// block stored at the start of the next period, 16 + ceil(5 L2_P / 4) + 1
// rows (the OR touches the row after the current one) never wrap onto an
// unstored dword.
#define L2_OUT 21u
#define L2_WMAX 4096u  // strings sorted at once by a workgroup
#define L2_NI 4        // transfers per period and direction, at most
#ifndef L2_PRIO
#define L2_PRIO 0      // A/B: wave issue priority by the group's longest string
#endif
#ifndef L2_TH
#define L2_TH 1u       // a period issues transfers once this many blocks wait (or one is urgent)
#endif

struct L2Shared {
  DecT<13> T;                             // the lookup at LDS offset 0
  uint32_t in[L2_WAVES][L2_IN * WAVE];    // input dword q (byte-swapped) of lane l at [64 (q mod L2_IN) + l]
  uint32_t out[L2_WAVES][L2_OUT * WAVE];  // output dword q at [64 (q mod L2_OUT) + l]
  uint16_t order[L2_WMAX];
  uint32_t hist[DL_CLASSES];
  uint32_t claimed;
};
static_assert(sizeof(L2Shared) <= 160u * 1024u, "lane decoder LDS");

// decode_batch_auto's slot of string s: 64 * (ceil(floor(8 x_s / 5) / 64) + s),
// x_s = off[s] - off[0]: 64-byte aligned, a multiple of 64 bytes, at least
// floor(8 E_s / 5) + 1 (lib/nghttp2_hd.c:2080-2082).
__device__ __host__ __forceinline__ uint64_t dl2_slot(uint32_t x, uint32_t s) {
  const uint64_t g = ((uint64_t)x * 8u) / 5u;
  return 64u * (((g + 63u) >> 6) + s);
}

__global__ __launch_bounds__(L2_NT) void k_decode_lanes2(const uint8_t *__restrict__ src,
                                                         const uint32_t *__restrict__ off, uint32_t n,
                                                         uint8_t *__restrict__ dst,
                                                         uint64_t dst_cap, uint32_t *__restrict__ dst_off,
                                                         int32_t *__restrict__ status,
                                                         uint16_t *__restrict__ fstate_out,
                                                         uint8_t *__restrict__ flags_out) {
  __shared__ L2Shared S;
  constexpr uint32_t LB = 13, G2 = 2u * 13u;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t q4 = lane >> 2, c4 = lane & 3u;  // as a loader: granule q4 of a transfer, piece c4
  lds_u32 *const inw = (lds_u32 *)S.in[wv];
  lds_u32 *const outw = (lds_u32 *)S.out[wv];
  lds_u32 *const inr = inw + lane;
  lds_u32 *const outr = outw + lane;
  const uint32_t off0 = __builtin_amdgcn_readfirstlane(off[0]);
  // this workgroup's strings: a contiguous range, balanced over the grid by
  // weight (encoded bytes + 32 per string; a 64-ary search over the offsets)
  uint32_t r0, r1;
  {
    const uint32_t nwg = gridDim.x, gw = blockIdx.x;
    const uint64_t wtot = (uint64_t)(off[n] - off0) + 32ull * n;
    auto first_at = [&](uint64_t target) -> uint32_t {  // smallest s with weight(s) >= target
      if (target == 0) return 0u;
      uint32_t lo = 0, hi = n;  // weight(lo) < target <= weight(hi)
      while (hi - lo > 1u) {
        const uint32_t step = (hi - lo + WAVE - 1u) / WAVE;
        const uint32_t c = min(lo + (lane + 1u) * step, hi);
        const uint64_t wc = (uint64_t)(off[c] - off0) + 32ull * c;
        const uint64_t ge = __ballot(wc >= target);  // (lane 63 or the clamp reaches hi)
        const uint32_t j = ge ? (uint32_t)__builtin_ctzll(ge) : WAVE - 1u;
        const uint32_t nhi = __builtin_amdgcn_readlane(c, j);
        lo = j ? __builtin_amdgcn_readlane(c, j - 1u) : lo;
        hi = nhi;
      }
      return hi;
    };
    r0 = first_at(wtot * gw / nwg);
    r1 = gw + 1u == nwg ? n : first_at(wtot * (gw + 1u) / nwg);
  }
  for (uint32_t r = 0; r < L2_OUT; ++r) outr[64u * r] = 0u;
  stage_dec_tables(S.T, L2_NT);
  const DecT<13> &T = S.T;
  DLS_INIT();
  const uint32_t src_lim = __builtin_amdgcn_readfirstlane(
      (uint32_t)u64min((((uint64_t)off[n] + 15u) & ~15ull) + 16u, (uint64_t)DL_OOB));
  auto uni_ptr = [](const void *p) -> void * {
    const uint64_t v = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (void *)(uintptr_t)(((uint64_t)hi << 32) | lo);
  };
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(uni_ptr(src), 0, (int)src_lim, 0x00020000);
  const uint32_t dst_lim = __builtin_amdgcn_readfirstlane((uint32_t)u64min(dst_cap, (uint64_t)DL_OOB));
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(uni_ptr(dst), 0, (int)dst_lim, 0x00020000);
  for (uint32_t w0 = r0; w0 < r1; w0 += L2_WMAX) {
    const uint32_t wn = min(L2_WMAX, r1 - w0), ngr = (wn + 63u) / 64u;
    __syncthreads();
    for (uint32_t c = threadIdx.x; c < DL_CLASSES; c += L2_NT) S.hist[c] = 0u;
    __syncthreads();
    constexpr uint32_t PT = (L2_WMAX + L2_NT - 1u) / L2_NT;
    uint32_t cls[PT];
#pragma unroll
    for (uint32_t u = 0; u < PT; ++u) {
      const uint32_t t = threadIdx.x + u * L2_NT;
      cls[u] = t < wn ? dl_class(off[w0 + t + 1] - off[w0 + t]) : 0u;
      if (t < wn) atomicAdd((uint32_t *)&S.hist[cls[u]], 1u);
    }
    __syncthreads();
    if (wv == 0) {
      const uint32_t h0 = S.hist[2u * lane], h1 = S.hist[2u * lane + 1u];
      const uint32_t inc = wave_incl_scan(h0 + h1);
      S.hist[2u * lane] = inc - h0 - h1;
      S.hist[2u * lane + 1u] = inc - h1;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < PT; ++u) {
      const uint32_t t = threadIdx.x + u * L2_NT;
      if (t < wn) S.order[atomicAdd((uint32_t *)&S.hist[cls[u]], 1u)] = (uint16_t)t;
    }
    if (threadIdx.x == 0) S.claimed = 0u;
    __syncthreads();
    auto claim = [&]() -> uint32_t {
      uint32_t gi = 0;
      if (lane == 0) gi = atomicAdd((uint32_t *)&S.claimed, 1u);
      return __builtin_amdgcn_readfirstlane(gi);
    };
    auto load_meta = [&](uint32_t gg) -> uint4 {  // {string, first byte, end}
      const uint32_t q = gg * 64u + lane;
      if (gg >= ngr || q >= wn) return make_uint4(DL_NONE, 0u, 0u, 0u);
      const uint32_t s = w0 + (uint32_t)S.order[q];
      return make_uint4(s, off[s], off[s + 1], 0u);
    };
    // A group's first input block and the first L2_IN - 16 dwords of the
    // next, prefetched during the previous group's tail: transfer h < 4
    // carries block b0 of owners 16 h .. 16 h + 15 (a quad per owner),
    // transfer 4 + t the first 32 bytes of block b0 + 1 of owners
    // 32 t .. 32 t + 31 (a lane pair per owner).
    static_assert(L2_IN == 24u, "prefetch: a block and 32 bytes");
    u32x4 pf[6];
    auto meta_span = [&](const uint4 &m, uint32_t &av, uint32_t &bv) {
      const bool ok = m.x != DL_NONE && m.z > m.y && m.y >= off0 && m.z - m.y < (1u << 28);
      av = ok ? m.y : 0u;
      bv = ok ? m.z : 0u;
    };
    auto prefetch = [&](const uint4 &m) {
      uint32_t av, bv;
      meta_span(m, av, bv);
#pragma unroll
      for (uint32_t h = 0; h < 4; ++h) {
        const uint32_t oa = __shfl(av, 16 * h + q4, 64), ob = __shfl(bv, 16 * h + q4, 64);
        const uint32_t at = ob > oa ? (oa & ~63u) + 16u * c4 : DL_OOB;
        pf[h] = __builtin_amdgcn_raw_buffer_load_b128(rd, at, 0, 0);
      }
#pragma unroll
      for (uint32_t t = 0; t < 2; ++t) {
        const uint32_t ow = 32u * t + (lane >> 1);
        const uint32_t oa = __shfl(av, ow, 64), ob = __shfl(bv, ow, 64);
        const uint32_t nb1 = (oa & ~63u) + 64u;
        const uint32_t at = ob > nb1 ? nb1 + 16u * (lane & 1u) : DL_OOB;
        pf[4 + t] = __builtin_amdgcn_raw_buffer_load_b128(rd, at, 0, 0);
      }
    };
    auto commit_pf = [&](const uint4 &m) {
      uint32_t av, bv;
      meta_span(m, av, bv);
      auto put4 = [&](uint32_t q, uint32_t ow, const u32x4 &v) {  // dwords q .. q + 3 of owner ow
        uint32_t r = q % L2_IN;
        inw[64u * r + ow] = __builtin_bswap32(v.x);
        r = r == L2_IN - 1u ? 0u : r + 1u;
        inw[64u * r + ow] = __builtin_bswap32(v.y);
        r = r == L2_IN - 1u ? 0u : r + 1u;
        inw[64u * r + ow] = __builtin_bswap32(v.z);
        r = r == L2_IN - 1u ? 0u : r + 1u;
        inw[64u * r + ow] = __builtin_bswap32(v.w);
      };
#pragma unroll
      for (uint32_t h = 0; h < 4; ++h) {
        const uint32_t ow = 16 * h + q4, oa = __shfl(av, ow, 64);
        put4(((oa & ~63u) >> 2) + 4u * c4, ow, pf[h]);
      }
#pragma unroll
      for (uint32_t t = 0; t < 2; ++t) {
        const uint32_t ow = 32u * t + (lane >> 1), oa = __shfl(av, ow, 64);
        put4(((oa & ~63u) >> 2) + 16u + 4u * (lane & 1u), ow, pf[4 + t]);
      }
    };
    uint32_t g = claim();
    uint4 mn = load_meta(g);
    prefetch(mn);
    DLS(0);
    while (g < ngr) {
      DLS_CNT(9);
      const uint4 mc = mn;
      commit_pf(mc);
      const bool have = mc.x != DL_NONE;
      const uint32_t i = have ? mc.x : 0u, a = mc.y, b = mc.z;
      const bool bad = have && (b < a || a < off0 || b - a >= (1u << 28));
      const bool act = have && !bad;
      const uint32_t E = act ? b - a : 0u;
#if L2_PRIO
      {  // groups of long strings set the kernel's tail: issue priority by length
        const uint32_t em = __builtin_amdgcn_readfirstlane(wave_max(E));
        if (em >= 512u) __builtin_amdgcn_s_setprio(3);
        else if (em >= 256u) __builtin_amdgcn_s_setprio(2);
        else if (em >= 128u) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      }
#endif
      const uint32_t gn = claim();
      mn = load_meta(gn);
      // ---- output slot [o, o + cap), 64-byte aligned
      const uint64_t s0 = dl2_slot(a - off0, i), s1 = act ? dl2_slot(b - off0, i + 1u) : s0;
      const uint32_t o = (uint32_t)u64min(s0, dst_cap);
      const bool slot_ovf = s1 > dst_cap;
      if (have) {
        dst_off[i] = o;
        if (i == n - 1u) dst_off[n] = (uint32_t)u64min(dl2_slot(off[n] - off0, n), dst_cap);
      }
      // ---- input: the ring holds dwords below in_end (16 b0 + L2_IN at
      // first); nreq = the next whole block to load, requested once the
      // dwords its rows held are taken (k >= 16 nreq - (L2_IN - 16))
      const uint32_t lastb = act && E ? (b - 1u) >> 6 : 0u;
      uint32_t nreq = (a >> 6) + 1u, in_end = 16u * (a >> 6) + L2_IN;
      bool reqd = false;  // block nreq in flight (committed next period)
      const uint32_t k0 = a >> 2, r8 = 8u * (a & 3u);
      const uint32_t kr0 = k0 % L2_IN, kr1 = kr0 == L2_IN - 1u ? 0u : kr0 + 1u;
      uint64_t bb = ((((uint64_t)inr[64u * kr0]) << 32) | inr[64u * kr1]) << r8;
      uint32_t nb = 64u - r8, k = k0 + 2u, kr = kr1 == L2_IN - 1u ? 0u : kr1 + 1u;  // kr: k's row
      uint32_t nxt = inr[64u * kr];
      uint32_t rem = 8u * E;
      // ---- output: P bits decoded; dword P >> 5 at ring row orow; st blocks stored
      uint32_t P = 0, st = 0, orow = (o >> 2) % L2_OUT;
#define L2_PUT(v, bits)                                                      \
  do {                                                                       \
    const uint64_t t_ = (uint64_t)(v) << (P & 31u);                          \
    const uint32_t r1_ = orow == L2_OUT - 1u ? 0u : orow + 1u;               \
    atomicOr((uint32_t *)&outr[64u * orow], (uint32_t)t_);                   \
    atomicOr((uint32_t *)&outr[64u * r1_], (uint32_t)(t_ >> 32));            \
    orow = ((P & 31u) + (bits)) >= 32u ? r1_ : orow;                         \
    P += (bits);                                                             \
  } while (0)
#define L2_REFILL()                                                      \
  do {                                                                   \
    const bool t_ = nb < 32u;                                            \
    bb |= (uint64_t)(t_ ? nxt : 0u) << ((32u - nb) & 63u);               \
    nb += t_ ? 32u : 0u;                                                 \
    k += t_ ? 1u : 0u;                                                   \
    kr = t_ ? (kr == L2_IN - 1u ? 0u : kr + 1u) : kr;                    \
    nxt = inr[64u * kr];                                                 \
  } while (0)
      // ---- transfers: rank the waiting lanes, one granule per loader quad
      auto rank_push = [&](bool need, uint32_t payload, uint32_t &cnt, uint32_t &rank) {
        const uint64_t m = __ballot(need);
        cnt = (uint32_t)__popcll(m);
        rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        (void)payload;
      };
      auto quad_get = [&](bool need, uint32_t rank, uint32_t ii, uint32_t payload) -> uint32_t {
        const bool push = need && rank >= 16u * ii && rank < 16u * ii + 16u;
        const uint32_t dl = push ? 4u * (rank - 16u * ii) : (lane | 1u);
        const uint32_t got = (uint32_t)__builtin_amdgcn_ds_permute((int)(4u * dl), (int)payload);
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)got, 0x00, 0xf, 0xf, true);  // quad_perm [0,0,0,0]
      };
      auto store_service = [&](bool need, bool urgent) {
        uint32_t cnt, rank;
        const uint32_t payload = (o + 64u * st) | lane;
        rank_push(need, payload, cnt, rank);
        if (cnt == 0u || (cnt < L2_TH && !__ballot(urgent))) return;
        const uint32_t ni = min((cnt + 15u) >> 4, (uint32_t)L2_NI);
#pragma unroll
        for (uint32_t ii = 0; ii < (uint32_t)L2_NI; ++ii) {
          if (ii < ni) {
            const uint32_t got = quad_get(need, rank, ii, payload);
            const bool valid = q4 + 16u * ii < cnt;
            const uint32_t ow = got & 63u, at = (got & ~63u) + 16u * c4;
            uint32_t rr = ((at >> 2)) % L2_OUT;
            u32x4 v;
            v.x = outw[64u * rr + ow];
            const uint32_t rr1 = rr == L2_OUT - 1u ? 0u : rr + 1u;
            v.y = outw[64u * rr1 + ow];
            const uint32_t rr2 = rr1 == L2_OUT - 1u ? 0u : rr1 + 1u;
            v.z = outw[64u * rr2 + ow];
            const uint32_t rr3 = rr2 == L2_OUT - 1u ? 0u : rr2 + 1u;
            v.w = outw[64u * rr3 + ow];
            if (valid) {
              outw[64u * rr + ow] = 0u;
              outw[64u * rr1 + ow] = 0u;
              outw[64u * rr2 + ow] = 0u;
              outw[64u * rr3 + ow] = 0u;
            }
            const uint32_t sa = valid && (uint64_t)at + 16u <= dst_cap ? at : DL_OOB;
            __builtin_amdgcn_raw_buffer_store_b128(v, wr, sa, 0, 0);
          }
        }
        if (need && rank < 16u * ni) ++st;
      };
      u32x4 stg[L2_NI];
      uint32_t sti[L2_NI];
      uint32_t nld = 0;
      auto load_service = [&](bool need, bool urgent) {
        uint32_t cnt, rank;
        const uint32_t payload = 64u * nreq | lane;
        rank_push(need, payload, cnt, rank);
        nld = 0;
        if (cnt == 0u || (cnt < L2_TH && !__ballot(urgent))) return;
        const uint32_t ni = min((cnt + 15u) >> 4, (uint32_t)L2_NI);
        nld = ni;
#pragma unroll
        for (uint32_t ii = 0; ii < (uint32_t)L2_NI; ++ii) {
          if (ii < ni) {
            const uint32_t got = quad_get(need, rank, ii, payload);
            const bool valid = q4 + 16u * ii < cnt;
            sti[ii] = valid ? got : DL_NONE;
            stg[ii] = __builtin_amdgcn_raw_buffer_load_b128(rd, valid ? (got & ~63u) + 16u * c4 : DL_OOB, 0, 0);
          }
        }
        if (need && rank < 16u * ni) reqd = true;
      };
      auto commit = [&]() {
#pragma unroll
        for (uint32_t ii = 0; ii < (uint32_t)L2_NI; ++ii) {
          if (ii < nld && sti[ii] != DL_NONE) {
            uint32_t r = ((sti[ii] & ~63u) >> 2) % L2_IN + 4u * c4;
            r = r >= L2_IN ? r - L2_IN : r;
            const uint32_t ow = sti[ii] & 63u;
            const u32x4 v = stg[ii];
            inw[64u * r + ow] = __builtin_bswap32(v.x);
            r = r == L2_IN - 1u ? 0u : r + 1u;
            inw[64u * r + ow] = __builtin_bswap32(v.y);
            r = r == L2_IN - 1u ? 0u : r + 1u;
            inw[64u * r + ow] = __builtin_bswap32(v.z);
            r = r == L2_IN - 1u ? 0u : r + 1u;
            inw[64u * r + ow] = __builtin_bswap32(v.w);
          }
        }
        nld = 0;
        if (reqd) {
          in_end = 16u * nreq + 16u;
          ++nreq;
          reqd = false;
        }
        nxt = inr[64u * kr];
      };
      bool failed = false, stopf = false;
      DLS(1);
      // ---- fast periods
      for (;;) {
        commit();
        const bool want = act && !failed && !stopf && rem >= G2;
        if (!__ballot(want)) break;
        DLS_CNT(10);
        store_service(act && (P >> 9) > st, true);  // every complete block (see L2_OUT)
        const bool all_in = nreq > lastb;
        const uint32_t avail = in_end - k;
        load_service(act && !all_in && k + (L2_IN - 16u) >= 16u * nreq, false);
        bool run = want && (all_in || avail >= 2u * L2_P) && (P >> 5) - 16u * st <= 15u;
        DLS(2);
#pragma unroll
        for (uint32_t p = 0; p < L2_P; ++p) {
          const uint32_t e1 = T.lut[(uint32_t)(bb >> 32) >> (32 - LB)];
          const uint32_t U1 = run ? E_USED(e1) : 0u;
          bb <<= U1;
          const uint32_t e2 = T.lut[(uint32_t)(bb >> 32) >> (32 - LB)];
          const uint32_t U2 = run ? E_USED(e2) : 0u;
          bb <<= U2;
          const uint32_t c1 = E_CNT8(e1);
          const uint32_t v = run ? ((e1 & 0xFFFFu) | ((e2 & 0xFFFFu) << c1)) : 0u;
          const uint32_t bits = run ? c1 + E_CNT8(e2) : 0u;
          L2_PUT(v, bits);
          nb -= U1 + U2;
          rem -= U1 + U2;
          L2_REFILL();
          const bool slow = run && e2 == 0u;  // a code longer than the lookup (an e1 of 0 stalls e2 too)
          if (__ballot(slow)) {
            if (slow) {
              const uint32_t e_ = slow_entry(T, (uint32_t)(bb >> 32), rem);
              if (e_ == 0xFFFFFFFFu) {
                failed = true;  // EOS: the FSM's sticky failure state
              } else if (E_L1(e_) > rem) {
                stopf = true;   // the string's tail: the careful steps take it
              } else {
                L2_PUT(e_ & 0xFFu, 8u);
                const uint32_t U_ = E_USED(e_);
                bb <<= U_;
                nb -= U_;
                rem -= U_;
                L2_REFILL();
              }
            }
          }
          run = run && !failed && !stopf && rem >= G2;
        }
        DLS(3);
      }
#undef L2_REFILL
      store_service(act && (P >> 9) > st, true);  // (room for the careful steps' bytes)
      prefetch(mn);  // the next group's first blocks, in flight over this one's tail
      // ---- careful steps: the last < 2 LB bits (or a long code at the tail)
      uint32_t t_bits = 0, t_win = 0;
      bool done = !act || failed;
      while (__ballot(!done)) {
        const uint32_t w = (uint32_t)(bb >> 32);
        const bool stop = done || rem == 0u;
        uint32_t e = T.lut[w >> (32 - LB)];
        const bool slow = e == 0u && !stop;
        if (__ballot(slow)) {
          if (slow) e = slow_entry(T, w, rem);
        }
        const bool eos = e == 0xFFFFFFFFu && !stop;
        const uint32_t L1 = E_L1(e), U = E_USED(e);
        const bool take1 = !stop && !eos && L1 <= rem;
        const bool take2 = take1 && E_CNT(e) == 2u && U <= rem;
        const bool tail = !stop && !eos && !take1;
        t_bits = tail ? rem : t_bits;
        t_win = tail ? w : t_win;
        const uint32_t adv = take2 ? U : (take1 ? L1 : 0u);
        if (take1) L2_PUT(e & (take2 ? 0xFFFFu : 0xFFu), take2 ? 16u : 8u);
        bb <<= adv;
        rem -= adv;
        failed = failed || eos;
        done = done || eos || !take1 || rem == 0u;
      }
#undef L2_PUT
      DLS(4);
      // ---- the rest of the output: every block with a decoded byte, whole
      while (__ballot(act && P > 512u * st)) store_service(act && P > 512u * st, true);
      if (have) {
        if (bad) {
          status[i] = NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
          if (fstate_out) {
            fstate_out[i] = 0u;
            flags_out[i] = 0u;
          }
        } else {
          dd_finish(T, failed, t_bits, t_win, P >> 3, slot_ovf, i, status, fstate_out, flags_out);
        }
      }
      g = gn;
      DLS(5);
    }
  }
  DLS_FLUSH();
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
    static unsigned long long z[4096][20];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z));
  }
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 4096 * 20);
}
#endif

template <uint32_t IP, int IW, int LB, uint32_t BI = 0>
static void launch_decode_items(const uint8_t *src, const uint32_t *src_off, uint32_t n,
                                uint8_t *dst, size_t dst_cap, uint32_t *dst_off,
                                int32_t *status, uint16_t *fstate, uint8_t *flags,
                                hipStream_t st) {
  hipLaunchKernelGGL((k_decode_items<IP, IW, LB, BI>),
                     dim3(persistent_grid<k_decode_items<IP, IW, LB, BI>, WAVE * IW, TASK_STR * IW>(n)),
                     dim3(WAVE * IW), 0, st, src, src_off, n, dst, (uint64_t)dst_cap, dst_off,
                     status, fstate, flags);
}

// piece = 64 / 40 / 32 (66..69: budgeted rounds) picks an instance; 0 picks
// by the batch's mean encoded string length, estimated from the pool size
// (dst_cap is normally nghttp2_amd_hd_huff_decode_bound(E, n) = 8 E / 5 +
// 4 n), so that most strings are one item.  Header strings of up to ~48
// bytes fit whole 64-byte items (no warm-up or item map) in budgeted rounds
// of at most 2304 input bytes, whose staging and output regions are sized
// for that budget instead of 64 full items: 16 waves per CU with the 13-bit
// lookup (config 2: 56.0 us, against 71-72 for <64, 8, 14> without a budget,
// 59.7 with a 2048-byte budget (2.3 % of config 2's tasks take two rounds),
// 55.7 / 56.7 with 2432 / 2560, 62.8 for the 14-bit lookup at 12 waves).
// Shorter ones too (the adversarial config 5: 158.6 us, against 164.3 in
// 32-byte items with the 20-byte warm-up; 261 in unbudgeted 64-byte items at
// 8 waves).  Longer values are cut into 40-byte pieces, also with the 13-bit
// lookup, whose 32 KB less LDS buys 16 waves per CU (measured: config 3 360
// vs 385 us for 40-byte items with the 14-bit lookup at 12 waves).  Every
// instance writes the same layout.
static int decode_items(const uint8_t *src, const uint32_t *src_off, uint32_t n, uint8_t *dst,
                        size_t dst_cap, uint32_t *dst_off, int32_t *status, uint16_t *fstate,
                        uint8_t *flags, void *stream, int piece) {
  hipStream_t st = (hipStream_t)stream;
  if (!dst_off) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (n == 0) return hip_rv(hipMemsetAsync(dst_off, 0, sizeof(uint32_t), st));
  if (!src || !src_off || !dst || !status) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if ((uint64_t)dst_cap > 0xFFFFFFFFull) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;  // uint32 offsets
  if (piece == 0) {
    const uint64_t est =
        (uint64_t)dst_cap > 4ull * n ? ((uint64_t)dst_cap - 4ull * n) * 5u / 8u : 0u;
    piece = est <= 48ull * n ? 68 : DD_PICK_LONG;
  }
#define DI_LAUNCH(P, W, B, ...) \
  launch_decode_items<P, W, B, ##__VA_ARGS__>(src, src_off, n, dst, dst_cap, dst_off, status, fstate, flags, st)
  switch (piece) {
    case 64: DI_LAUNCH(64u, 8, 14); break;
    case 66: DI_LAUNCH(64u, 12, 14, 2048u); break;  // budgeted rounds
    case 67: DI_LAUNCH(64u, 16, 13, 2048u); break;
    case 68: DI_LAUNCH(64u, 16, 13, 2304u); break;
    case 69: DI_LAUNCH(32u, 16, 14, 1280u); break;
    case 40: DI_LAUNCH(40u, 16, 13); break;
    case 32: DI_LAUNCH(32u, 16, 13); break;
#if DD_PICK_LONG != 40  // A/B builds: 40-byte pieces at fewer waves (LDS left for other kernels)
    case 42: DI_LAUNCH(40u, 12, 13); break;
    case 43: DI_LAUNCH(40u, 13, 13); break;
    case 45: DI_LAUNCH(40u, 14, 13); break;
#endif
#if DD_XINST  // A/B builds: the other lookup width at the same pieces; other budgets
    case 70: DI_LAUNCH(64u, 16, 13, 2560u); break;
    case 71: DI_LAUNCH(64u, 16, 13, 2432u); break;
    case 65: DI_LAUNCH(64u, 10, 13); break;
    case 41: DI_LAUNCH(40u, 12, 14); break;
    case 44: DI_LAUNCH(44u, 15, 13); break;
    case 33: DI_LAUNCH(32u, 14, 14); break;
    case 36: DI_LAUNCH(36u, 13, 14); break;
    case 30: DI_LAUNCH(30u, 15, 14); break;
#endif
    default: return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  }
#undef DI_LAUNCH
  return hip_rv(hipGetLastError());
}

// The lane decoder: AUTO slots (written to dst_off) or the caller's slots.
// Each resident workgroup takes a window of ceil(n / grid) strings (whole
// groups of 64) and, when `sort`, decodes it in length order.
template <bool AUTO>
static int decode_lanes(const uint8_t *src, const uint32_t *src_off, uint32_t n, uint8_t *dst,
                        size_t dst_cap, uint32_t *dst_off, int32_t *status, uint16_t *fstate,
                        uint8_t *flags, void *stream, bool sort) {
  hipStream_t st = (hipStream_t)stream;
  if (!dst_off) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (n == 0) return AUTO ? hip_rv(hipMemsetAsync(dst_off, 0, sizeof(uint32_t), st)) : 0;
  if (!src || !src_off || !dst || !status) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if ((fstate == nullptr) != (flags == nullptr)) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (AUTO && (uint64_t)dst_cap > 0xFFFFFFFFull) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  const uint32_t grid = persistent_grid<k_decode_lanes<AUTO>, DL_NT, 64>(n);
  const uint32_t win = (uint32_t)((((uint64_t)n + grid - 1u) / grid + 63u) & ~63ull);
  hipLaunchKernelGGL((k_decode_lanes<AUTO>), dim3(grid), dim3(DL_NT), 0, st, src, src_off, n, win,
                     sort ? 1u : 0u, dst, (uint64_t)dst_cap, dst_off, status, fstate, flags);
  return hip_rv(hipGetLastError());
}

static int decode_lanes2(const uint8_t *src, const uint32_t *src_off, uint32_t n, uint8_t *dst,
                         size_t dst_cap, uint32_t *dst_off, int32_t *status, uint16_t *fstate,
                         uint8_t *flags, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!dst_off) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (n == 0) return hip_rv(hipMemsetAsync(dst_off, 0, sizeof(uint32_t), st));
  if (!src || !src_off || !dst || !status) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if ((fstate == nullptr) != (flags == nullptr)) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if ((uint64_t)dst_cap > 0xFFFFFFFFull) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  const uint32_t grid = persistent_grid<k_decode_lanes2, L2_NT, 64>(n);
  hipLaunchKernelGGL(k_decode_lanes2, dim3(grid), dim3(L2_NT), 0, st, src, src_off, n, dst,
                     (uint64_t)dst_cap, dst_off, status, fstate, flags);
  return hip_rv(hipGetLastError());
}

extern "C" {

// Lane decoder, A/B entry: mode bit 0 = the caller's slots (decode_batch
// semantics; dst_cap ignored), bit 1 = string order (no length sort).
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd__decode_batch_lanes(const uint8_t *src, const uint32_t *src_off,
                                                          uint32_t n, uint8_t *dst, size_t dst_cap,
                                                          uint32_t *dst_off, int32_t *status,
                                                          uint16_t *fstate, uint8_t *flags,
                                                          void *stream, int mode) {
  const bool sort = !(mode & 2);
  if (mode & 4)
    return decode_lanes2(src, src_off, n, dst, dst_cap, dst_off, status, fstate, flags, stream);
  if (mode & 1)
    return decode_lanes<false>(src, src_off, n, dst, dst_cap, dst_off, status, fstate, flags,
                               stream, sort);
  return decode_lanes<true>(src, src_off, n, dst, dst_cap, dst_off, status, fstate, flags, stream,
                            sort);
}
#if DL_STAMPS
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd__dl_stamps(void *out, int reset) {
  if (reset) {
    static unsigned long long z[2048][12];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_dl_stamps), z, sizeof(z));
  }
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dl_stamps), sizeof(unsigned long long) * 2048 * 12);
}
#endif

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

size_t nghttp2_amd_hd_huff_encode_workspace_size(uint64_t raw_bytes, uint32_t n) {
  const size_t slots = (size_t)enc_piece_slot(0, 0, 0) + raw_bytes / ENC_PIECE + n + 1u;
  return nghttp2_amd_hd_huff_workspace_size(n) + ((slots * sizeof(uint16_t) + 15u) & ~(size_t)15u);
}

int nghttp2_amd_hd_huff_encode_count_batch(const uint8_t *src, const uint32_t *src_off,
                                           uint32_t n, uint32_t *enc_len, void *stream) {
  if (n == 0) return 0;
  if (!src || !src_off || !enc_len) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(k_enc_count, dim3(ntiles_for(n)), dim3(WG), 0, (hipStream_t)stream, src,
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
  uint32_t *tiles = (uint32_t *)workspace;
  hipLaunchKernelGGL(k_enc_count, dim3(nt), dim3(WG), 0, st, src, src_off, n, dst_off, tiles, 1);
  hipLaunchKernelGGL(k_encode, dim3(nt), dim3(WG), 0, st, src, src_off, n, dst,
                     (uint64_t)dst_cap, dst_off, (const uint32_t *)tiles);
  return hip_rv(hipGetLastError());
}

// The round-1 encode kernels (byte-aligned heads inside chunks), kept for
// A/B measurement only.
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd__encode_batch_r1(const uint8_t *src, const uint32_t *src_off,
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
  hipLaunchKernelGGL(k_enc_count_r1, dim3(nt), dim3(WG), 0, st, src, src_off, n, dst_off, tiles,
                     (uint16_t *)nullptr, 1);
  hipLaunchKernelGGL(k_encode_r1, dim3(nt), dim3(WG), 0, st, src, src_off, n, dst,
                     (uint64_t)dst_cap, dst_off, (const uint32_t *)tiles);
  return hip_rv(hipGetLastError());
}

size_t nghttp2_amd_hd_emit_strings_bound(uint64_t raw_bytes, uint32_t n) {
  // a 32-bit length takes at most 6 prefix bytes (1 + ceil(32 / 7))
  const uint64_t b = raw_bytes + 6u * (uint64_t)n + 16u;
  return (size_t)((b + 15u) & ~(uint64_t)15u);
}

// workspace: [tile scratch][encoded offsets (n + 1)][encoded pool]
static size_t a256(size_t x) { return (x + 255u) & ~(size_t)255u; }
size_t nghttp2_amd_hd_emit_strings_workspace_size(uint64_t raw_bytes, uint32_t n) {
  return a256(nghttp2_amd_hd_huff_workspace_size(n)) + a256(4u * ((size_t)n + 1u)) +
         a256(nghttp2_amd_hd_huff_encode_bound(raw_bytes, n));
}

int nghttp2_amd_hd_emit_strings_batch(const uint8_t *src, const uint32_t *src_off, uint32_t n,
                                      uint64_t raw_bytes, uint8_t *dst, size_t dst_cap,
                                      uint32_t *dst_off, void *workspace, size_t workspace_size,
                                      void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!dst_off) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (n == 0) return hip_rv(hipMemsetAsync(dst_off, 0, sizeof(uint32_t), st));
  if (!src || !src_off || !dst || !workspace) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (((uintptr_t)workspace & 255u) ||
      workspace_size < nghttp2_amd_hd_emit_strings_workspace_size(raw_bytes, n) ||
      dst_cap < nghttp2_amd_hd_emit_strings_bound(raw_bytes, n))
    return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  uint8_t *w = (uint8_t *)workspace;
  uint32_t *tiles = (uint32_t *)w;
  const size_t ws_t = a256(nghttp2_amd_hd_huff_workspace_size(n));
  uint32_t *eoff = (uint32_t *)(w + ws_t);
  uint8_t *epool = w + ws_t + a256(4u * ((size_t)n + 1u));
  const size_t ecap = nghttp2_amd_hd_huff_encode_bound(raw_bytes, n);
  int rv = nghttp2_amd_hd_huff_encode_batch(src, src_off, n, epool, ecap, eoff, tiles, ws_t, stream);
  if (rv) return rv;
  const uint32_t nt = ntiles_for(n);
  hipLaunchKernelGGL(k_frame_len, dim3(nt), dim3(WG), 0, st, src_off, (const uint32_t *)eoff, n,
                     dst_off, tiles);
  hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(SCAN_WG), 0, st, tiles, nt, dst_off + n);
  hipLaunchKernelGGL(k_scan_apply, dim3(nt), dim3(WG), 0, st, dst_off, n, (const uint32_t *)tiles);
  hipLaunchKernelGGL(k_frame_copy, dim3(nt), dim3(WG), 0, st, src, src_off, (const uint8_t *)epool,
                     (const uint32_t *)eoff, n, dst, (uint64_t)dst_cap, (const uint32_t *)dst_off);
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
  hipLaunchKernelGGL(k_decode<false>, dim3(persistent_grid<k_decode<false>, DEC_NT, TASK_STR * DEC_WAVES>(n)), dim3(DEC_NT), 0,
                     (hipStream_t)stream, src, src_off, n, dst, (uint64_t)0,
                     (uint32_t *)dst_off, status, fstate, flags);
  return hip_rv(hipGetLastError());
}

int nghttp2_amd_hd_huff_decode_batch_auto(const uint8_t *src, const uint32_t *src_off,
                                          uint32_t n, uint8_t *dst, size_t dst_cap,
                                          uint32_t *dst_off, int32_t *status,
                                          uint16_t *fstate, uint8_t *flags, void *stream) {
  return decode_items(src, src_off, n, dst, dst_cap, dst_off, status, fstate, flags, stream, 0);
}

// decode_batch_auto with a chosen instance (piece bytes 64, 40 or 32), for
// the parity tests and A/B measurement.
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd__decode_batch_items(const uint8_t *src,
                                                          const uint32_t *src_off, uint32_t n,
                                                          uint8_t *dst, size_t dst_cap,
                                                          uint32_t *dst_off, int32_t *status,
                                                          uint16_t *fstate, uint8_t *flags,
                                                          void *stream, int piece) {
  return decode_items(src, src_off, n, dst, dst_cap, dst_off, status, fstate, flags, stream,
                      piece);
}

// The byte-balanced-piece dense decoder (pieces cross string ends), kept for
// A/B measurement only.
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd__decode_batch_pieces(const uint8_t *src,
                                                           const uint32_t *src_off, uint32_t n,
                                                           uint8_t *dst, size_t dst_cap,
                                                           uint32_t *dst_off, int32_t *status,
                                                           uint16_t *fstate, uint8_t *flags,
                                                           void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!dst_off) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (n == 0) return hip_rv(hipMemsetAsync(dst_off, 0, sizeof(uint32_t), st));
  if (!src || !src_off || !dst || !status) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if ((uint64_t)dst_cap > 0xFFFFFFFFull) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(k_decode_dense,
                     dim3(persistent_grid<k_decode_dense, DD_NT, TASK_STR * DD_WAVES>(n)),
                     dim3(DD_NT), 0, st, src, src_off, n, dst, (uint64_t)dst_cap, dst_off, status,
                     fstate, flags);
  return hip_rv(hipGetLastError());
}

// The round-1 engine-slot decoder (one launch, a 4-byte aligned slot of
// auto_slot() bytes per string), kept for A/B measurement only.
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd__decode_batch_slots(const uint8_t *src,
                                                          const uint32_t *src_off, uint32_t n,
                                                          uint8_t *dst, size_t dst_cap,
                                                          uint32_t *dst_off, int32_t *status,
                                                          uint16_t *fstate, uint8_t *flags,
                                                          void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!dst_off) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if (n == 0) return hip_rv(hipMemsetAsync(dst_off, 0, sizeof(uint32_t), st));
  if (!src || !src_off || !dst || !status) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  if ((uint64_t)dst_cap > 0xFFFFFFFFull) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  hipLaunchKernelGGL(k_decode<true>, dim3(persistent_grid<k_decode<true>, DEC_NT, TASK_STR * DEC_WAVES>(n)), dim3(DEC_NT), 0, st, src, src_off,
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
