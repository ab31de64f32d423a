/*
 * nghttp2_amd_hd_testing.h -- test hooks of the batched HPACK front-ends.
 *
 * Not part of the drop-in boundary: the parity tests use these to force the
 * code paths a small test batch would not take on its own (the two switches
 * are process-wide settings read at the next nghttp2_amd_hd_deflate_blocks
 * call), and the bench its copy ceiling.
 */
#ifndef NGHTTP2_AMD_HD_TESTING_H
#define NGHTTP2_AMD_HD_TESTING_H

#include <stdint.h>

#ifndef NGHTTP2_AMD_EXTERN
#define NGHTTP2_AMD_EXTERN __attribute__((visibility("default")))
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* The next n GPU calls of the deflater fail as a HIP error would (0: none):
 * the deflaters of the batch must turn bad, as on INSUFF_BUFSIZE. */
NGHTTP2_AMD_EXTERN void nghttp2_amd_hd__test_fail_deflate_gpu(int n);

/* Batches of at least n header names take the GPU name-token kernel (the
 * default threshold keeps small batches on the host). */
NGHTTP2_AMD_EXTERN void nghttp2_amd_hd__set_gpu_names_min(uint32_t n);

/* Device-to-device streaming copy of `bytes` bytes (16-byte aligned, a
 * multiple of 64) on `stream`: four 16-byte loads in flight per lane over a
 * grid-stride loop.  bench.py times it as the measured HBM ceiling that the
 * roofline's frac_vs_copy is taken against. */
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd__copy_calib(void *dst, const void *src, size_t bytes,
                                                  void *stream);

/* Bounds-checked debug build (the library compiled with HD_BOUNDS=1,
 * lib/libnghttp2_amd_hd_bounds.so): waits for the device, then reports in
 * *site the first out-of-bounds index the hot-path kernels recorded since
 * the last call (0: none; 0x1xx encode, 0x2xx decode -- the sites are listed
 * in DESIGN.md) and clears the record; *site == 0x5E1F7E57 on entry first
 * runs a self-test kernel that records site 0x1FF.  Returns 0, a negative
 * error, or 1 in the product build, which compiles no checks. */
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd__bounds_check(uint32_t *site);

#ifdef __cplusplus
}
#endif

#endif /* NGHTTP2_AMD_HD_TESTING_H */
