// chain_probe.hip -- how much a second independent lookup chain per lane buys
// the decode's pair loop, before building it into k_decode_items.
//
// Each lane decodes 40-byte items of a Huffman stream (config-3-like bytes:
// 85 % cookie alphabet, 15 % printable) staged once in its wave's LDS, with
// the product's pair loop shape: a register window (alignbit over three
// staged words), the 13-bit two-symbol lookup in LDS, a second lookup at the
// first entry's used bits, four byte stores into the lane's LDS output
// region, the next word prefetched from LDS.  CH = 1: one item per lane (the
// product); CH = 2: two items per lane stepped in one loop.  Waves per CU are
// set by the workgroup size (one workgroup per CU: LDS padded past half).
// Codes past the lookup advance 13 bits and emit nothing (about 1 % of
// steps; the product's slow path is not the question here).
// Prints decoded bytes per microsecond for each (CH, waves) point.
//
// Build: hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-sched-strategy=max-ilp \
//        -o chain_probe chain_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

namespace dev {
#define HD_TBL static __device__
#include "../../../nghttp2_amd/csrc/hd_huff_tables.inc"
#undef HD_TBL
}  // namespace dev
namespace host {
#define HD_TBL static
#include "../../../nghttp2_amd/csrc/hd_huff_tables.inc"
#undef HD_TBL
}  // namespace host

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) u32x2 lds_u32x2;

constexpr uint32_t IP = 40;          // item bytes
constexpr uint32_t OB = 72;          // output region per item (di_rb(40))
constexpr uint32_t LUT_WORDS = 8192; // 13-bit lookup

#define E_USED(e) ((e) >> 27)
#define E_CNT8(e) (((e) >> 10) & 0x18u)

template <int CH>
struct Chain {
  uint32_t A, B, N, nq;
  int32_t kw, nG;
  lds_u8 *p;
};

// W waves per workgroup, CH chains per lane, R repeats of the wave's round.
// V (CH = 1 only; what the pair loop's LDS time goes to): 0 the product's
// shape; 1 no output stores; 2 one dword store per pair (bytes gathered in a
// 64-bit register, the dword stored when full); 3 lookups made bank-conflict
// free (each lane of a 32-lane group on its own bank; wrong symbols, the
// same step count on average); 4 no prefetch read of the next staged word;
// 5 the pair's raw entries stored as one aligned 8-byte record; 6 its four
// symbol bytes as one aligned 4-byte record (both: compaction not included)
template <int CH, int V = 0>
__global__ void k_probe(const uint32_t *__restrict__ enc_words, uint32_t nwords, uint32_t R,
                        uint32_t *__restrict__ out_bytes) {
  extern __shared__ uint32_t smem[];
  lds_u32 *lut = (lds_u32 *)smem;
  const uint32_t W = blockDim.x >> 6, wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  constexpr uint32_t IBW = (64u * IP * CH) / 4u + 16u;  // staged words per wave
  constexpr uint32_t OBB = 64u * OB * CH;
  lds_u32 *ib = lut + LUT_WORDS + wv * (IBW + OBB / 4u);
  lds_u8 *ob = (lds_u8 *)(ib + IBW);
  for (uint32_t i = threadIdx.x; i < LUT_WORDS; i += blockDim.x) lut[i] = dev::hd_huff_lut13[i];
  // the wave's staged stream: a slice of the encoded words (bytes in
  // big-endian words, as the product stages them)
  const uint32_t g = (blockIdx.x * W + wv) * 997u;
  for (uint32_t i = lane; i < IBW; i += 64u) ib[i] = enc_words[(g + i) % nwords];
  __syncthreads();
  uint32_t total = 0;
  for (uint32_t r = 0; r < R; ++r) {
    Chain<CH> c[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const uint32_t item = lane + 64u * j;
      const uint32_t bp = 8u * IP * item + 1u + (r & 7u);  // (bp >= 1)
      const uint32_t stop = 8u * IP * (item + 1u) - 26u;
      c[j].kw = (int32_t)(bp - 1u) >> 5;
      c[j].A = ib[c[j].kw];
      c[j].B = ib[c[j].kw + 1];
      c[j].N = ib[c[j].kw + 2];
      c[j].nq = ~(bp - 1u);
      c[j].nG = ~((int32_t)stop - 1);
      c[j].p = ob + OB * item;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_setprio(1);
    if (CH == 1 && V >= 7) {
      // V 7: the bytes of pair i gathered into a 64-bit register and stored
      // as whole dwords, done while pair i + 1's first lookup is in flight
      // (software-pipelined); V 8: the next staged words read two at a time,
      // every second pair; V 9: both
      Chain<CH> &x = c[0];
      uint64_t acc = 0;
      uint32_t nb = 0, pe1 = 0, pe2 = 0, N1 = 0, par = 0;
      lds_u32 *q = (lds_u32 *)x.p;
      if (V >= 8) N1 = ib[(uint32_t)x.kw + 3u];
      while ((int32_t)x.nq >= x.nG) {
        const uint32_t w = __builtin_amdgcn_alignbit(x.A, x.B, x.nq);
        const uint32_t e1 = lut[w >> 19];
        // (the gather below after the lookup's issue, not before it)
        __builtin_amdgcn_sched_barrier(0);
        if (V != 8) {
          const uint32_t c1 = E_CNT8(pe1);
          const uint32_t b = __builtin_amdgcn_perm(0u, pe1, 0x0C0C0200u) |
                             (__builtin_amdgcn_perm(0u, pe2, 0x0C0C0200u) << c1);
          acc |= (uint64_t)b << nb;
          nb += c1 + E_CNT8(pe2);
          *q = (uint32_t)acc;
          const bool full = nb >= 32u;
          q += full ? 1 : 0;
          acc = full ? acc >> 32 : acc;
          nb -= full ? 32u : 0u;
        }
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t U1 = e1 ? E_USED(e1) : 13u;
        const uint32_t e2 = lut[(w << U1) >> 19];
        const uint32_t U2 = e2 ? E_USED(e2) : 13u;
        if (V == 8) {
          x.p[0] = (uint8_t)e1;
          x.p[1] = (uint8_t)(e1 >> 16);
          x.p += E_CNT8(e1) >> 3;
          x.p[0] = (uint8_t)e2;
          x.p[1] = (uint8_t)(e2 >> 16);
          x.p += E_CNT8(e2) >> 3;
        }
        pe1 = e1;
        pe2 = e2;
        const uint32_t u = U1 + U2;
        const bool t = u > (x.nq & 31u);
        x.nq -= u;
        x.A = t ? x.B : x.A;
        x.B = t ? x.N : x.B;
        x.kw += t ? 1 : 0;
        if (V >= 8) {
          // words kw + 2, kw + 3 held in N, N1; read two every second pair
          // (two pairs cross at most two words: 52 bits)
          x.N = t ? N1 : x.N;
          par ^= 1u;
          if (par == 0u) {
            const uint32_t k2 = (uint32_t)x.kw + 2u;
            x.N = ib[k2];
            N1 = ib[k2 + 1u];
          }
        } else {
          x.N = ib[(uint32_t)x.kw + 2u];
        }
      }
      if (V != 8) {
        const uint32_t c1 = E_CNT8(pe1);
        nb += c1 + E_CNT8(pe2);
        x.p = (lds_u8 *)q + (nb >> 3);
      }
    } else     if (CH == 1) {
      Chain<CH> &x = c[0];
      uint64_t acc = 0;
      uint32_t nb = 0, npair = 0;
      while ((int32_t)x.nq >= x.nG) {
        const uint32_t w = __builtin_amdgcn_alignbit(x.A, x.B, x.nq);
        const uint32_t i1 = V == 3 ? (((w >> 19) & ~31u) | (lane & 31u)) : (w >> 19);
        const uint32_t e1 = lut[i1];
        const uint32_t U1 = e1 ? E_USED(e1) : 13u;
        const uint32_t i2 = V == 3 ? ((((w << U1) >> 19) & ~31u) | (lane & 31u)) : ((w << U1) >> 19);
        const uint32_t e2 = lut[i2];
        const uint32_t U2 = e2 ? E_USED(e2) : 13u;
        if (V == 1) {
          x.p += (E_CNT8(e1) + E_CNT8(e2)) >> 3;
        } else if (V == 10) {
          // the pair's 2-4 symbol bytes packed and stored as one dword at the
          // (unaligned) byte position; the next store overwrites the rest
          const uint32_t c1 = E_CNT8(e1);
          const uint32_t b = __builtin_amdgcn_perm(0u, e1, 0x0C0C0200u) |
                             (__builtin_amdgcn_perm(0u, e2, 0x0C0C0200u) << c1);
          *(lds_u32 *)x.p = b;
          x.p += (c1 + E_CNT8(e2)) >> 3;
        } else if (V == 11) {
          // 4-byte record per pair (V 6) plus the two entries' symbol counts
          // gathered in a 64-bit register, 4 bits a pair
          *(lds_u32 *)(ob + OB * lane + 4u * (npair & 15u)) = __builtin_amdgcn_perm(e2, e1, 0x06040200u);
          const uint32_t cc = ((e1 >> 13) & 3u) | (((e2 >> 13) & 3u) << 2);
          acc |= (uint64_t)cc << (4u * (npair & 15u));
          ++npair;
          x.p += (E_CNT8(e1) + E_CNT8(e2)) >> 3;
        } else if (V == 5 || V == 6) {
          // the pair's two raw entries as one 8-byte record (compacted to
          // bytes later, outside the loop); V 6: one 4-byte record (the
          // symbol bytes, 0 and 2 of each entry)
          if (V == 5) *(lds_u32x2 *)(ob + OB * lane + 8u * (npair & 7u)) = u32x2{e1, e2};
          else *(lds_u32 *)(ob + OB * lane + 4u * (npair & 15u)) = __builtin_amdgcn_perm(e2, e1, 0x06040200u);
          ++npair;
          x.p += (E_CNT8(e1) + E_CNT8(e2)) >> 3;
        } else if (V == 2) {
          // both entries' bytes (0 and 2 of each) contiguous, then into acc
          const uint32_t b1 = __builtin_amdgcn_perm(0u, e1, 0x0C0C0200u);
          const uint32_t b2 = __builtin_amdgcn_perm(0u, e2, 0x0C0C0200u);
          const uint32_t c1 = E_CNT8(e1);
          const uint64_t b = (uint64_t)b1 | ((uint64_t)b2 << c1);
          acc |= b << nb;
          nb += c1 + E_CNT8(e2);
          *(lds_u32 *)x.p = (uint32_t)acc;
          const bool full = nb >= 32u;
          x.p += full ? 4 : 0;
          acc = full ? acc >> 32 : acc;
          nb -= full ? 32u : 0u;
        } else {
          x.p[0] = (uint8_t)e1;
          x.p[1] = (uint8_t)(e1 >> 16);
          x.p += E_CNT8(e1) >> 3;
          x.p[0] = (uint8_t)e2;
          x.p[1] = (uint8_t)(e2 >> 16);
          x.p += E_CNT8(e2) >> 3;
        }
        const uint32_t u = U1 + U2;
        const bool t = u > (x.nq & 31u);
        x.nq -= u;
        x.A = t ? x.B : x.A;
        x.B = t ? x.N : x.B;
        x.kw += t ? 1 : 0;
        if (V == 4) x.N = x.A ^ x.kw;
        else x.N = ib[(uint32_t)x.kw + 2u];
      }
      if (V == 2) x.p += nb >> 3;
      if (V == 11) total += (uint32_t)(acc >> 60);  // (keeps the mask live)
    } else {
      // both chains step together while either runs; a finished chain's
      // step takes no bits and its pointer does not move
      for (;;) {
        bool any = false;
#pragma unroll
        for (int j = 0; j < CH; ++j) any |= (int32_t)c[j].nq >= c[j].nG;
        if (!any) break;
        uint32_t w[CH], e1[CH], e2[CH];
#pragma unroll
        for (int j = 0; j < CH; ++j) {
          w[j] = __builtin_amdgcn_alignbit(c[j].A, c[j].B, c[j].nq);
          e1[j] = lut[w[j] >> 19];
        }
#pragma unroll
        for (int j = 0; j < CH; ++j) {
          const uint32_t U1 = e1[j] ? E_USED(e1[j]) : 13u;
          e2[j] = lut[(w[j] << U1) >> 19];
        }
#pragma unroll
        for (int j = 0; j < CH; ++j) {
          Chain<CH> &x = c[j];
          const bool on = (int32_t)x.nq >= x.nG;
          const uint32_t U1 = e1[j] ? E_USED(e1[j]) : 13u;
          const uint32_t U2 = e2[j] ? E_USED(e2[j]) : 13u;
          x.p[0] = (uint8_t)e1[j];
          x.p[1] = (uint8_t)(e1[j] >> 16);
          lds_u8 *p2 = x.p + (E_CNT8(e1[j]) >> 3);
          p2[0] = (uint8_t)e2[j];
          p2[1] = (uint8_t)(e2[j] >> 16);
          p2 += E_CNT8(e2[j]) >> 3;
          x.p = on ? p2 : x.p;
          const uint32_t u = on ? U1 + U2 : 0u;
          const bool t = u > (x.nq & 31u);
          x.nq -= u;
          x.A = t ? x.B : x.A;
          x.B = t ? x.N : x.B;
          x.kw += t ? 1 : 0;
          x.N = ib[(uint32_t)x.kw + 2u];
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);
#pragma unroll
    for (int j = 0; j < CH; ++j) total += (uint32_t)(c[j].p - (ob + OB * (lane + 64u * j)));
  }
  out_bytes[blockIdx.x * blockDim.x + threadIdx.x] = total;
}

int main(int argc, char **argv) {
  const uint32_t R = argc > 1 ? atoi(argv[1]) : 64;
  // config-3-like bytes, Huffman-encoded on the host
  const char *cookie = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/=;,-_%";
  const size_t ncookie = strlen(cookie);
  std::vector<uint8_t> enc;
  uint64_t acc = 0;
  int nb = 0;
  uint32_t s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return s >> 8; };
  while (enc.size() < (16u << 20)) {
    const uint32_t c = (rnd() % 100u) < 85u ? (uint8_t)cookie[rnd() % ncookie] : 0x20u + rnd() % 95u;
    const uint32_t len = host::hd_huff_enc_len[c], code = host::hd_huff_enc_code[c] >> (32u - len);
    acc = (acc << len) | code;  // (len <= 30)
    nb += len;
    while (nb >= 8) {
      enc.push_back((uint8_t)(acc >> (nb - 8)));
      nb -= 8;
    }
  }
  std::vector<uint32_t> words(enc.size() / 4);
  for (size_t i = 0; i < words.size(); ++i)
    words[i] = (uint32_t)enc[4 * i] << 24 | (uint32_t)enc[4 * i + 1] << 16 | (uint32_t)enc[4 * i + 2] << 8 | enc[4 * i + 3];
  uint32_t *d_w, *d_out;
  CK(hipMalloc(&d_w, words.size() * 4));
  CK(hipMemcpy(d_w, words.data(), words.size() * 4, hipMemcpyHostToDevice));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipMalloc(&d_out, (size_t)cus * 1024 * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](auto kern, int CH, int W) {
    const size_t ibw = (64u * IP * CH) / 4u + 16u, obb = 64u * OB * CH;
    size_t lds = 4u * LUT_WORDS + W * (4u * ibw + obb);
    if (lds < 82u * 1024u) lds = 82u * 1024u;  // one workgroup per CU
    if (lds > 160u * 1024u) {
      printf("CH=%d W=%2d: %zu B of LDS, does not fit\n", CH, W, lds);
      return;
    }
    CK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(kern, dim3(cus), dim3(64 * W), lds, 0, d_w, (uint32_t)words.size(), R, d_out);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int k = 0; k < 5; ++k) {
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(kern, dim3(cus), dim3(64 * W), lds, 0, d_w, (uint32_t)words.size(), R, d_out);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      best = ms < best ? ms : best;
    }
    std::vector<uint32_t> o((size_t)cus * 64 * W);
    CK(hipMemcpy(o.data(), d_out, o.size() * 4, hipMemcpyDeviceToHost));
    double bytes = 0;
    for (uint32_t v : o) bytes += v;
    printf("CH=%d W=%2d lds=%6zu  %.3f ms  decoded %.1f MB  %.1f B/us  (%.1f B/us per chain-wave slot)\n", CH, W,
           lds, best, bytes / 1e6, bytes / (best * 1e3), bytes / (best * 1e3) / (CH * W));
  };
  for (int W : {4, 8, 12, 16}) run(k_probe<1>, 1, W);
  for (int W : {12, 16}) {
    printf("variant 1 (no output stores): ");
    run(k_probe<1, 1>, 1, W);
    printf("variant 2 (one dword store per pair): ");
    run(k_probe<1, 2>, 1, W);
    printf("variant 3 (conflict-free lookups): ");
    run(k_probe<1, 3>, 1, W);
    printf("variant 4 (no prefetch read): ");
    run(k_probe<1, 4>, 1, W);
    printf("variant 5 (one 8-byte record per pair): ");
    run(k_probe<1, 5>, 1, W);
    printf("variant 6 (one 4-byte record per pair): ");
    run(k_probe<1, 6>, 1, W);
    printf("variant 10 (one unaligned dword store per pair): ");
    run(k_probe<1, 10>, 1, W);
    printf("variant 11 (4-byte record + count mask): ");
    run(k_probe<1, 11>, 1, W);
    printf("variant 7 (pipelined dword gather): ");
    run(k_probe<1, 7>, 1, W);
    printf("variant 8 (two-word refill every 2nd pair): ");
    run(k_probe<1, 8>, 1, W);
    printf("variant 9 (7 + 8): ");
    run(k_probe<1, 9>, 1, W);
  }
  for (int W : {4, 6, 8, 10}) run(k_probe<2>, 2, W);
  return 0;
}
