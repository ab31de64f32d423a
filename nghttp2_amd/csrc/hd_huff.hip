// hd_huff.hip -- MI355X (gfx950) HPACK Huffman engine: kernels + C ABI.
//
// Replaces the reference's scalar loops in lib/nghttp2_hd_huffman.c
// (encode_count :34-43, encode :45-104, decode :111-143) for batches of
// independent header strings laid out SoA in HBM (see
// include/nghttp2_amd_hd.h and DESIGN.md).
//
// Kernel set (all integer/table work, no MFMA):
//   k_enc_count   per-string encoded length (sum of code lengths) + per-tile
//                 sums for the offset scan
//   k_scan_tiles  exclusive scan of the tile sums (one workgroup)
//   k_scan_apply  in-tile exclusive scan -> offsets (decode slots)
//   k_encode      in-tile scan -> encoded offsets, then MSB-first bit packing
//                 with EOS-prefix padding (lib/nghttp2_hd_huffman.c:95-101)
//   k_decode      nibble-stepped FSM (lib/nghttp2_hd_huffman.c:122-133) over
//                 the 257x16 transition table staged in LDS
//
// Work layout: a workgroup (256 lanes) owns a tile of TILE consecutive
// strings; lane t owns strings [tile*TILE + t*SPL, +SPL), whose input bytes
// and output bytes are each one contiguous stream, so every lane reads its
// input with aligned 16-byte loads and writes whole aligned 32-bit words
// except at its two stream ends.  Tables are staged in LDS once per
// workgroup.
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

#define WG 256
#define SPL 16
#define TILE (WG * SPL)
#define SCAN_WG 1024

#define HUFF_ACCEPTED 0x01u
#define HUFF_SYM 0x02u

// ---------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------

// Inclusive scan across the 64 lanes of a wave.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

// Exclusive scan across a workgroup of NT threads; returns the exclusive
// prefix, writes the workgroup total to *total.  `sm` needs NT/64 words.
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

// Byte stream reader over [p, end) of the pool with aligned 16-byte loads.
// The pool is readable up to align_up(end, 16) (API contract).
struct ByteIn {
  const uint8_t *base;
  uint32_t pos;     // absolute byte index of the next byte
  uint32_t chunk;   // absolute index of the loaded chunk (multiple of 16)
  uint4 v;
  __device__ __forceinline__ void init(const uint8_t *b, uint32_t p) {
    base = b;
    pos = p;
    chunk = 0xFFFFFFFFu;
  }
  __device__ __forceinline__ uint32_t get() {
    uint32_t c = pos & ~15u;
    if (c != chunk) {
      chunk = c;
      v = *reinterpret_cast<const uint4 *>(base + c);
    }
    uint32_t k = pos & 15u;
    uint32_t w = (k < 8) ? ((k < 4) ? v.x : v.y) : ((k < 12) ? v.z : v.w);
    ++pos;
    return (w >> ((k & 3u) * 8u)) & 0xFFu;
  }
};

// Byte stream writer: packs bytes into aligned 32-bit words; the (up to)
// partial words at the two ends of a stream go out as single bytes, so two
// lanes whose streams share a word never overwrite each other's bytes.
struct ByteOut {
  uint8_t *p;   // address of the first pending byte
  uint32_t w;   // pending bytes, little-endian from p
  uint32_t k;   // pending byte count (0..3)
  __device__ __forceinline__ void init(uint8_t *q) {
    p = q;
    w = 0;
    k = 0;
  }
  __device__ __forceinline__ void flush() {
    for (uint32_t i = 0; i < k; ++i) p[i] = (uint8_t)(w >> (8 * i));
    p += k;
    w = 0;
    k = 0;
  }
  __device__ __forceinline__ void put(uint32_t b) {
    w |= b << (8 * k);
    ++k;
    if ((((uintptr_t)p + k) & 3u) == 0) {
      if (k == 4) {
        *reinterpret_cast<uint32_t *>(p) = w;
        p += 4;
        w = 0;
        k = 0;
      } else {
        flush();
      }
    }
  }
};

// ---------------------------------------------------------------------------
// encode: lengths + tile sums   (lib/nghttp2_hd_huffman.c:34-43)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(WG) void k_enc_count(const uint8_t *__restrict__ src,
                                                  const uint32_t *__restrict__ off,
                                                  uint32_t n,
                                                  uint32_t *__restrict__ out_len,
                                                  uint32_t *__restrict__ tile_sums) {
  __shared__ uint32_t lenT[256];
  __shared__ uint32_t red[WG / 64];
  lenT[threadIdx.x] = dev::hd_huff_enc_len[threadIdx.x];
  __syncthreads();
  const uint32_t s0 = blockIdx.x * TILE + threadIdx.x * SPL;
  uint32_t lane_sum = 0;
  if (s0 < n) {
    const uint32_t s1 = min(s0 + SPL, n);
    ByteIn in;
    uint32_t a = off[s0];
    in.init(src, a);
    for (uint32_t s = s0; s < s1; ++s) {
      const uint32_t b = off[s + 1];
      uint32_t bits = 0;
      for (uint32_t p = a; p < b; ++p) bits += lenT[in.get()];
      const uint32_t e = (bits + 7u) >> 3;
      if (out_len) out_len[s] = e;
      lane_sum += e;
      a = b;
    }
  }
  if (tile_sums) {
    uint32_t tot;
    block_excl_scan<WG>(lane_sum, red, &tot);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
  }
}

// decode slots: cap_i = floor(8 E_i / 5) + 1 (lib/nghttp2_hd_huffman.h:76-78)
__global__ __launch_bounds__(WG) void k_slot_len(const uint32_t *__restrict__ off,
                                                 uint32_t n,
                                                 uint32_t *__restrict__ out_len,
                                                 uint32_t *__restrict__ tile_sums) {
  __shared__ uint32_t red[WG / 64];
  const uint32_t s0 = blockIdx.x * TILE + threadIdx.x * SPL;
  uint32_t lane_sum = 0;
  for (uint32_t j = 0; j < SPL; ++j) {
    const uint32_t s = s0 + j;
    if (s < n) {
      const uint32_t e = off[s + 1] - off[s];
      const uint32_t c = (uint32_t)(((uint64_t)e * 8u) / 5u) + 1u;
      out_len[s] = c;
      lane_sum += c;
    }
  }
  uint32_t tot;
  block_excl_scan<WG>(lane_sum, red, &tot);
  if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
}

// Exclusive scan of ntiles tile sums in place; writes the grand total to
// *grand (== offsets[n]).
__global__ __launch_bounds__(SCAN_WG) void k_scan_tiles(uint32_t *__restrict__ tile_sums,
                                                        uint32_t ntiles,
                                                        uint32_t *__restrict__ grand) {
  __shared__ uint32_t sm[SCAN_WG / 64];
  uint32_t carry = 0;
  for (uint32_t base = 0; base < ntiles; base += SCAN_WG) {
    const uint32_t i = base + threadIdx.x;
    const uint32_t v = (i < ntiles) ? tile_sums[i] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl_scan<SCAN_WG>(v, sm, &tot);
    if (i < ntiles) tile_sums[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) *grand = carry;
}

// In-place: offs[i] holds a length on entry, the exclusive prefix on exit.
__device__ __forceinline__ uint32_t tile_offsets(uint32_t *offs, uint32_t n,
                                                 const uint32_t *tile_prefix,
                                                 uint32_t *red, uint32_t loc[SPL]) {
  const uint32_t s0 = blockIdx.x * TILE + threadIdx.x * SPL;
  uint32_t lane_sum = 0;
#pragma unroll
  for (int j = 0; j < SPL; ++j) {
    const uint32_t s = s0 + j;
    loc[j] = (s < n) ? offs[s] : 0u;
    lane_sum += loc[j];
  }
  uint32_t tot;
  uint32_t run = tile_prefix[blockIdx.x] + block_excl_scan<WG>(lane_sum, red, &tot);
#pragma unroll
  for (int j = 0; j < SPL; ++j) {
    const uint32_t s = s0 + j;
    const uint32_t len = loc[j];
    loc[j] = run;
    if (s < n) offs[s] = run;
    run += len;
  }
  return run;  // end offset of the lane's last string
}

__global__ __launch_bounds__(WG) void k_scan_apply(uint32_t *__restrict__ offs, uint32_t n,
                                                   const uint32_t *__restrict__ tile_prefix) {
  __shared__ uint32_t red[WG / 64];
  uint32_t loc[SPL];
  tile_offsets(offs, n, tile_prefix, red, loc);
}

// ---------------------------------------------------------------------------
// encode: bit packing    (lib/nghttp2_hd_huffman.c:45-104)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(WG) void k_encode(const uint8_t *__restrict__ src,
                                               const uint32_t *__restrict__ off,
                                               uint32_t n, uint8_t *__restrict__ dst,
                                               uint64_t dst_cap,
                                               uint32_t *__restrict__ dst_off,
                                               const uint32_t *__restrict__ tile_prefix) {
  __shared__ uint2 codeT[256];
  __shared__ uint32_t red[WG / 64];
  codeT[threadIdx.x] = make_uint2(dev::hd_huff_enc_code[threadIdx.x],
                                  dev::hd_huff_enc_len[threadIdx.x]);
  uint32_t loc[SPL];
  const uint32_t end_out = tile_offsets(dst_off, n, tile_prefix, red, loc);
  __syncthreads();
  const uint32_t s0 = blockIdx.x * TILE + threadIdx.x * SPL;
  if (s0 >= n) return;
  if ((uint64_t)end_out > dst_cap) return;  // never write past the pool
  const uint32_t s1 = min(s0 + SPL, n);
  ByteIn in;
  uint32_t a = off[s0];
  in.init(src, a);
  ByteOut out;
  out.init(dst + loc[0]);
  for (uint32_t s = s0; s < s1; ++s) {
    const uint32_t b = off[s + 1];
    uint64_t acc = 0;  // MSB-aligned pending bits
    uint32_t nb = 0;
    for (uint32_t p = a; p < b; ++p) {
      const uint2 e = codeT[in.get()];
      acc |= (uint64_t)e.x << (32 - nb);
      nb += e.y;
      while (nb >= 8) {
        out.put((uint32_t)(acc >> 56));
        acc <<= 8;
        nb -= 8;
      }
    }
    if (nb) {  // pad with the EOS prefix (all ones)
      out.put((uint32_t)(acc >> 56) | ((1u << (8 - nb)) - 1u));
    }
    a = b;
  }
  out.flush();
}

// ---------------------------------------------------------------------------
// decode: nibble FSM    (lib/nghttp2_hd_huffman.c:111-143)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(WG) void k_decode(const uint8_t *__restrict__ src,
                                               const uint32_t *__restrict__ off,
                                               uint32_t n, uint8_t *__restrict__ dst,
                                               const uint32_t *__restrict__ dst_off,
                                               int32_t *__restrict__ status,
                                               uint16_t *__restrict__ fstate_out,
                                               uint8_t *__restrict__ flags_out) {
  __shared__ uint32_t fsm[257 * 16];
  for (uint32_t i = threadIdx.x; i < 257 * 16; i += WG) fsm[i] = dev::hd_huff_fsm[i];
  __syncthreads();
  const uint32_t s0 = blockIdx.x * TILE + threadIdx.x * SPL;
  if (s0 >= n) return;
  const uint32_t s1 = min(s0 + SPL, n);
  ByteIn in;
  uint32_t a = off[s0];
  in.init(src, a);
  for (uint32_t s = s0; s < s1; ++s) {
    const uint32_t b = off[s + 1];
    const uint32_t o0 = dst_off[s];
    const uint32_t cap = dst_off[s + 1] - o0;
    ByteOut out;
    out.init(dst + o0);
    uint32_t t = (HUFF_ACCEPTED << 16);  // {fstate 0, flags ACCEPTED}
    uint32_t w = 0;
    bool overflow = false;
    for (uint32_t p = a; p < b; ++p) {
      const uint32_t c = in.get();
      t = fsm[(t & 0x1FFu) * 16u + (c >> 4)];
      if (t & (HUFF_SYM << 16)) {
        if (w < cap) out.put(t >> 24); else overflow = true;
        ++w;
      }
      t = fsm[(t & 0x1FFu) * 16u + (c & 15u)];
      if (t & (HUFF_SYM << 16)) {
        if (w < cap) out.put(t >> 24); else overflow = true;
        ++w;
      }
    }
    out.flush();
    const uint32_t flags = (t >> 16) & 0xFFu;
    int32_t st;
    if (overflow) st = NGHTTP2_AMD_ERR_BUFFER_ERROR;
    else if (!(flags & HUFF_ACCEPTED)) st = NGHTTP2_AMD_ERR_HEADER_COMP;
    else st = (int32_t)w;
    status[s] = st;
    if (fstate_out) fstate_out[s] = (uint16_t)(t & 0xFFFFu);
    if (flags_out) flags_out[s] = (uint8_t)flags;
    a = b;
  }
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
static inline uint32_t ntiles_for(uint32_t n) { return (n + TILE - 1) / TILE; }

static int hip_rv(hipError_t e) {
  if (e == hipSuccess) return 0;
  fprintf(stderr, "nghttp2_amd_hd: HIP error %s\n", hipGetErrorString(e));
  return NGHTTP2_AMD_ERR_FATAL;
}

extern "C" {

const char *nghttp2_amd_hd_version(void) { return "nghttp2_amd_hd 0.1.0 gfx950"; }

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

size_t nghttp2_amd_hd_huff_workspace_size(uint32_t n) {
  return ((size_t)ntiles_for(n) + 16u) * sizeof(uint32_t);
}

int nghttp2_amd_hd_huff_encode_count_batch(const uint8_t *src, const uint32_t *src_off,
                                           uint32_t n, uint32_t *enc_len, void *stream) {
  if (n == 0) return 0;
  if (!src || !src_off || !enc_len) return NGHTTP2_AMD_ERR_INVALID_ARGUMENT;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_enc_count, dim3(ntiles_for(n)), dim3(WG), 0, st, src, src_off, n,
                     enc_len, (uint32_t *)nullptr);
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
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_decode, dim3(ntiles_for(n)), dim3(WG), 0, st, src, src_off, n, dst,
                     dst_off, status, fstate, flags);
  return hip_rv(hipGetLastError());
}

}  // extern "C"
