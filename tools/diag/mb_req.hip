// Microbenchmark: cost of per-lane scattered 16-byte loads / stores against
// the same bytes in fewer, wider requests (G lanes on one string: pairs,
// quads, or a whole coalesced 1 KiB), with a part of the lanes active, at the
// lane decoder's shape: 16 waves per CU, one workgroup per CU, 64 "strings"
// per wave each streamed sequentially.  "res" cases fold every address into
// 1 MiB (L2-resident: the memory pipe alone, no HBM); the others stream from
// HBM.  Question it answers: is the lane decoder's memory time set by
// instructions, by lines touched per instruction, or by bytes?
//
// build: hipcc -O3 --offload-arch=gfx950 -o tools/diag/mb_req tools/diag/mb_req.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// G lanes per string per instruction (1, 2, 4, 64); 64 / G strings per
// instruction, rotating over the wave's 64 strings; a string advances 16 G
// bytes per visit.  Lanes of 1 / act of the string groups are active.
template <int STORE>
__global__ __launch_bounds__(1024) void k_req(uint8_t *buf, uint32_t periods, uint32_t G, uint32_t act,
                                              uint32_t span, uint64_t amask, uint32_t *sink) {
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t wbase = ((uint64_t)blockIdx.x * 16u + wv) * 64u * span;  // the wave's 64 strings
  const uint32_t per = 64u / G;  // strings per instruction
  const uint32_t rot = 64u / per;
  u32x4 acc = {0, 0, 0, 0};
  u32x4 val = {lane, wv, blockIdx.x, 7u};
#pragma unroll 8
  for (uint32_t p = 0; p < periods; ++p) {
    const uint32_t grp = lane / G;
    const uint32_t s = (p % rot) * per + grp;
    const uint32_t visit = p / rot;
    const uint64_t a = (wbase + (uint64_t)s * span + (uint64_t)visit * 16u * G + 16u * (lane % G)) & amask;
    if (((grp + p) % act) == 0u) {
      if (STORE) {
        *(u32x4 *)(buf + a) = val;
        val += 1u;
      } else {
        acc ^= *(const u32x4 *)(buf + a);
      }
    }
  }
  if (!STORE && (acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1u;
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint32_t P = 256;           // instructions per wave
  const uint32_t span = 16u * P;    // a string never wraps (G = 1, act = 1 is the longest walk)
  const size_t bytes = (size_t)cus * 16 * 64 * span;
  uint8_t *buf;
  uint32_t *sink;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 1, bytes));
  hipEvent_t ea, eb;
  CK(hipEventCreate(&ea));
  CK(hipEventCreate(&eb));
  const int Gs[4] = {1, 2, 4, 64};
  const int acts[3] = {1, 3, 8};
  for (int st = 0; st < 2; ++st)
    for (int res = 1; res >= 0; --res)
      for (int gi = 0; gi < 4; ++gi)
        for (int ai = 0; ai < 3; ++ai) {
          const uint32_t G = Gs[gi], act = acts[ai];
          if (G == 64 && act != 1) continue;
          const uint64_t amask = res ? ((1ull << 20) - 16u) : ~15ull;
          float best = 1e30f;
          for (int r = 0; r < 4; ++r) {
            CK(hipEventRecord(ea));
            if (st)
              hipLaunchKernelGGL(k_req<1>, dim3(cus), dim3(1024), 0, 0, buf, P, G, act, span, amask, sink);
            else
              hipLaunchKernelGGL(k_req<0>, dim3(cus), dim3(1024), 0, 0, buf, P, G, act, span, amask, sink);
            CK(hipEventRecord(eb));
            CK(hipEventSynchronize(eb));
            float ms;
            CK(hipEventElapsedTime(&ms, ea, eb));
            if (ms < best) best = ms;
          }
          const double instr_cu = 16.0 * P;              // wave-instructions per CU
          const double lanes = 64.0 / act;               // active lanes per instruction
          const double lines = (G == 64 ? 8.0 : 64.0 / G) / act;  // 64 B-granule groups approx
          const double cyc = best * 1e-3 * 2.1e9;
          printf("{\"op\": \"%s\", \"res\": %d, \"G\": %u, \"act\": %u, \"us\": %.1f, \"GBps\": %.0f, "
                 "\"cyc_per_instr\": %.1f, \"reqs_per_instr\": %.1f, \"cyc_per_req\": %.2f}\n",
                 st ? "st" : "ld", res, G, act, best * 1e3, cus * instr_cu * lanes * 16.0 / (best * 1e-3) / 1e9,
                 cyc / instr_cu, lines, cyc / instr_cu / lines);
          fflush(stdout);
        }
  CK(hipFree(buf));
  return 0;
}
