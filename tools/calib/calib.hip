// WRITE_SIZE / FETCH_SIZE calibration on known byte counts (gfx950).
// Each kernel moves exactly BYTES bytes; run under rocprofv3 --pmc.
#include <hip/hip_runtime.h>
#include <stdio.h>
#define BYTES (64u << 20)
__global__ void st_dword(uint32_t *p) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < BYTES / 4; i += gridDim.x * blockDim.x) p[i] = i;
}
__global__ void st_dwordx4(uint4 *p) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < BYTES / 16; i += gridDim.x * blockDim.x) p[i] = make_uint4(i, i, i, i);
}
__global__ void st_byte(uint8_t *p) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < BYTES; i += gridDim.x * blockDim.x) p[i] = (uint8_t)i;
}
__global__ void ld_dword(const uint32_t *p, uint32_t *out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x, acc = 0;
  for (; i < BYTES / 4; i += gridDim.x * blockDim.x) acc += p[i];
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ void ld_dwordx4(const uint4 *p, uint32_t *out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x, acc = 0;
  for (; i < BYTES / 16; i += gridDim.x * blockDim.x) { uint4 v = p[i]; acc += v.x ^ v.y ^ v.z ^ v.w; }
  if (acc == 0x12345678u) out[0] = acc;
}
// tile pattern: each workgroup copies a TILE-byte region that starts at a
// 4-byte-aligned (not line-aligned) offset, like the decode's staged slots
template <int ALIGN>
__global__ void st_tiles(uint32_t *p, uint32_t tile_words) {
  const uint32_t base = blockIdx.x * tile_words + (ALIGN == 4 ? (blockIdx.x * 7u) % 32u : 0u);
  for (uint32_t i = threadIdx.x; i < tile_words; i += blockDim.x) p[base + i] = i;
}
int main() {
  void *a, *b;
  if (hipMalloc(&a, BYTES) || hipMalloc(&b, BYTES)) return 1;
  hipMemset(a, 1, BYTES);
  for (int r = 0; r < 3; ++r) {
    st_dword<<<2048, 256>>>((uint32_t *)b);
    st_dwordx4<<<2048, 256>>>((uint4 *)b);
    st_byte<<<2048, 256>>>((uint8_t *)b);
    ld_dword<<<2048, 256>>>((const uint32_t *)a, (uint32_t *)b);
    ld_dwordx4<<<2048, 256>>>((const uint4 *)a, (uint32_t *)b);
    // 13 KB tiles covering ~60 MB: 4-byte-misaligned vs 128-byte aligned starts
    st_tiles<4><<<4600, 256>>>((uint32_t *)b, 3328);
    st_tiles<128><<<4600, 256>>>((uint32_t *)b, 3328);
  }
  hipDeviceSynchronize();
  printf("calib done: %u bytes per kernel\n", BYTES);
  return 0;
}
