// Probe: LDS accesses at byte addresses (ds_write_b16 / ds_read_b32 at odd
// offsets) -- do they act on the addressed bytes (unaligned mode)?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef __attribute__((address_space(3))) uint8_t l8;
typedef __attribute__((address_space(3))) uint16_t l16;
typedef __attribute__((address_space(3))) uint32_t l32;
__global__ void k(uint32_t *out) {
  __shared__ __attribute__((aligned(16))) uint8_t b[256];
  const uint32_t t = threadIdx.x;
  for (uint32_t i = t; i < 256; i += 64) b[i] = (uint8_t)(i * 7 + 1);
  __syncthreads();
  // each lane writes 0xBEEF at byte offset 2 t + 1 (odd) ... lanes 0..31 only
  l16 *w = (l16 *)((l8 *)b + 2 * t + 1);
  if (t < 32) *w = (uint16_t)(0xBE00u | t);
  __syncthreads();
  uint32_t bytes = 0;
  for (int j = 0; j < 4; ++j) bytes |= (uint32_t)b[4 * t + j] << (8 * j);
  out[t] = bytes;
  __syncthreads();
  const l32 *r = (const l32 *)((l8 *)b + t + 1);  // read at t + 1
  out[64 + t] = *r;
}
int main() {
  uint32_t *d;
  uint32_t h[128];
  if (hipMalloc(&d, 512) != hipSuccess) return 2;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 3; }
  if (hipMemcpy(h, d, 512, hipMemcpyDeviceToHost) != hipSuccess) return 4;
  // expected, on the host
  uint8_t b[256];
  for (int i = 0; i < 256; ++i) b[i] = (uint8_t)(i * 7 + 1);
  for (int t = 0; t < 32; ++t) { b[2 * t + 1] = (uint8_t)t; b[2 * t + 2] = 0xBE; }
  int bad_w = 0, bad_r = 0;
  for (int t = 0; t < 64; ++t) {
    uint32_t e = 0, e2 = 0;
    for (int j = 0; j < 4; ++j) e |= (uint32_t)b[4 * t + j] << (8 * j);
    for (int j = 0; j < 4; ++j) e2 |= (uint32_t)b[t + 1 + j] << (8 * j);
    bad_w += h[t] != e;
    bad_r += h[64 + t] != e2;
  }
  printf("unaligned ds_write_b16 mismatches %d, unaligned ds_read_b32 mismatches %d\n", bad_w, bad_r);
  printf("lane1 read %08x want %08x\n", h[65], (uint32_t)(b[2] | b[3] << 8 | b[4] << 16 | b[5] << 24));
  return 0;
}
