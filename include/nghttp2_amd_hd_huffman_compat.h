/*
 * nghttp2_amd_hd_huffman_compat.h -- link-level drop-in for nghttp2's
 * internal HPACK Huffman API (lib/nghttp2_hd.h:385-440).
 *
 * libnghttp2_amd_hd.so exports the five functions below with the reference's
 * exact names, signatures and semantics, so an nghttp2 build can drop
 * lib/nghttp2_hd_huffman.c + lib/nghttp2_hd_huffman_data.c and link this
 * library instead.  Every call runs on the GPU (a batch of
 * one string through the same kernels as the batched API): correct for any
 * caller, but latency-bound per call -- high-rate callers use the batched
 * API in nghttp2_amd_hd.h.
 *
 * The structs restate the reference's layouts field for field (they are the
 * ABI the functions take); inside an nghttp2 build define
 * NGHTTP2_AMD_HAVE_NGHTTP2_TYPES and include the reference headers first.
 *
 * nghttp2_hd_huff_encode appends to a chained nghttp2_bufs through
 * nghttp2_bufs_addb, which libnghttp2 provides (lib/nghttp2_buf.c:372); the
 * engine binds it weakly and returns NGHTTP2_ERR_BUFFER_ERROR if no
 * implementation is linked.
 */
#ifndef NGHTTP2_AMD_HD_HUFFMAN_COMPAT_H
#define NGHTTP2_AMD_HD_HUFFMAN_COMPAT_H

#include <stddef.h>
#include <stdint.h>

#ifndef NGHTTP2_AMD_EXTERN
#define NGHTTP2_AMD_EXTERN __attribute__((visibility("default")))
#endif

#ifdef __cplusplus
extern "C" {
#endif

#ifndef NGHTTP2_AMD_HAVE_NGHTTP2_TYPES
typedef ptrdiff_t nghttp2_ssize; /* lib/includes/nghttp2/nghttp2.h:84 */

/* lib/nghttp2_buf.h:39-53 */
typedef struct {
  uint8_t *begin;
  uint8_t *end;
  uint8_t *pos;
  uint8_t *last;
  uint8_t *mark;
} nghttp2_buf;

/* lib/nghttp2_buf.h:122-132 */
typedef struct nghttp2_buf_chain nghttp2_buf_chain;
struct nghttp2_buf_chain {
  nghttp2_buf_chain *next;
  nghttp2_buf buf;
};

/* lib/nghttp2_buf.h:134-155 (mem is the nghttp2_mem allocator, opaque here) */
typedef struct {
  nghttp2_buf_chain *head;
  nghttp2_buf_chain *cur;
  void *mem;
  size_t chunk_length;
  size_t max_chunk;
  size_t chunk_used;
  size_t chunk_keep;
  size_t offset;
} nghttp2_bufs;

/* lib/nghttp2_hd_huffman.h:56-60 */
typedef struct {
  uint16_t fstate;
  uint8_t flags;
} nghttp2_hd_huff_decode_context;
#endif /* NGHTTP2_AMD_HAVE_NGHTTP2_TYPES */

/* lib/nghttp2_hd.h:394 -- encoded length incl. EOS-prefix padding.  If the
 * engine fails (no device, no memory) it returns len, so emit_string
 * (lib/nghttp2_hd.c:1011) takes the raw form rather than framing a
 * zero-length Huffman literal. */
NGHTTP2_AMD_EXTERN size_t nghttp2_hd_huff_encode_count(const uint8_t *src, size_t len);

/* lib/nghttp2_hd.h:408-409 -- appends the encoding of src to bufs; 0 or
 * NGHTTP2_ERR_BUFFER_ERROR (-502) / NGHTTP2_ERR_NOMEM (-901) from the bufs
 * layer, with the same bytes written before the error as the reference. */
NGHTTP2_AMD_EXTERN int nghttp2_hd_huff_encode(nghttp2_bufs *bufs, const uint8_t *src, size_t srclen);

/* lib/nghttp2_hd.h:411 */
NGHTTP2_AMD_EXTERN void nghttp2_hd_huff_decode_context_init(nghttp2_hd_huff_decode_context *ctx);

/* lib/nghttp2_hd.h:432-434 -- decodes a (possibly partial, fin == 0) chunk
 * from the carried context; writes to buf->last (caller guarantees room for
 * srclen * 8 / 5 bytes); returns srclen, or NGHTTP2_ERR_HEADER_COMP (-523)
 * when fin and the final state does not accept. */
NGHTTP2_AMD_EXTERN nghttp2_ssize nghttp2_hd_huff_decode(nghttp2_hd_huff_decode_context *ctx, nghttp2_buf *buf,
                                     const uint8_t *src, size_t srclen, int fin);

/* lib/nghttp2_hd.h:440 -- nonzero when EOS was decoded (state 0x100) */
NGHTTP2_AMD_EXTERN int nghttp2_hd_huff_decode_failure_state(nghttp2_hd_huff_decode_context *ctx);

#ifdef __cplusplus
}
#endif

#endif /* NGHTTP2_AMD_HD_HUFFMAN_COMPAT_H */
