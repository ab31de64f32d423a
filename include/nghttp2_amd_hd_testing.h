/*
 * nghttp2_amd_hd_testing.h -- test hooks of the batched HPACK front-ends.
 *
 * Not part of the drop-in boundary: the parity tests use these to force the
 * code paths a small test batch would not take on its own.  Both are
 * process-wide settings read at the next nghttp2_amd_hd_deflate_blocks call.
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

#ifdef __cplusplus
}
#endif

#endif /* NGHTTP2_AMD_HD_TESTING_H */
