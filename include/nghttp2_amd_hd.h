/*
 * nghttp2_amd_hd.h -- C ABI of the MI355X-native HPACK Huffman engine.
 *
 * This is the drop-in boundary for nghttp2's HPACK Huffman hot path
 * (lib/nghttp2_hd_huffman.c + lib/nghttp2_hd_huffman_data.c in the
 * reference).  Plain C: pointers, sizes and ints only.  HIP streams are
 * passed as `void *` (a hipStream_t; NULL = the default stream).
 *
 * Two groups of entry points:
 *
 *  1. Batched, device-resident API (nghttp2_amd_hd_huff_*_batch).  N
 *     independent header strings in SoA form: one contiguous byte pool plus
 *     uint32 offsets[N+1] (string i = pool[off[i] .. off[i+1])).  All
 *     pointers are device pointers (hipMalloc'd or HBM-resident torch
 *     storage).  Calls are asynchronous on `stream`.  This is what the
 *     batched drivers (replacing src/deflatehd.cc / src/inflatehd.cc) and
 *     an integration under emit_string / hd_inflate_read_huff bind.
 *
 *  2. Link-level replacements of the reference's internal Huffman API
 *     (lib/nghttp2_hd.h:394-440) -- see nghttp2_amd_hd_huffman_compat.h.
 *
 * Pool requirements (device API): pool base pointers 16-byte aligned; the
 * source pool readable up to align_up(off[N], 16) + 16 bytes (kernels load
 * aligned 16-byte words and unaligned 4-byte windows).  Offsets are uint32, so one batch's pool is
 * < 4 GiB; shard larger sets (multi-GPU).
 *
 * Error convention: 0 on success or a negative nghttp2_error code
 * (lib/includes/nghttp2/nghttp2.h:278-459).  Per-string decode results are
 * reported in a status array, never by the return value.
 */
#ifndef NGHTTP2_AMD_HD_H
#define NGHTTP2_AMD_HD_H

#include <stddef.h>
#include <stdint.h>

#ifndef NGHTTP2_AMD_EXTERN
#define NGHTTP2_AMD_EXTERN __attribute__((visibility("default")))
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* nghttp2_error values used on this path (lib/includes/nghttp2/nghttp2.h) */
#define NGHTTP2_AMD_ERR_INVALID_ARGUMENT (-501) /* nghttp2.h:278 */
#define NGHTTP2_AMD_ERR_BUFFER_ERROR (-502)     /* nghttp2.h:282 */
#define NGHTTP2_AMD_ERR_HEADER_COMP (-523)      /* nghttp2.h:378 */
#define NGHTTP2_AMD_ERR_INSUFF_BUFSIZE (-525)   /* nghttp2.h:386 */
#define NGHTTP2_AMD_ERR_FATAL (-900)            /* nghttp2.h:451 (HIP error) */
#define NGHTTP2_AMD_ERR_NOMEM (-901)            /* nghttp2.h:455 */

/* dst_off[n] after nghttp2_amd_hd_huff_encode_batch when the batch's encoded
 * total does not fit min(dst_cap, 0xFFFFFFFE): offsets are uint32, so such a
 * batch must be split (no offset of it is valid, no byte was written at or
 * past dst_cap). */
#define NGHTTP2_AMD_OFF_OVERFLOW 0xFFFFFFFFu

/* Decode-context flag bits (lib/nghttp2_hd_huffman.h:35-37). */
#define NGHTTP2_AMD_HUFF_ACCEPTED 0x01u
#define NGHTTP2_AMD_HUFF_SYM 0x02u
/* Failure (EOS decoded) state id (lib/nghttp2_hd_huffman.h:44-48). */
#define NGHTTP2_AMD_HUFF_FAIL_STATE 0x100u

/* Library version string, e.g. "nghttp2_amd_hd 0.1.0 gfx950". */
NGHTTP2_AMD_EXTERN const char *nghttp2_amd_hd_version(void);

/* Copies the engine's Huffman tables out in the reference's struct layouts
 * so a caller can check them against lib/nghttp2_hd_huffman_data.c without a
 * GPU: sym_out receives huff_sym_table (257 x {u32 nbits, u32 code} = 2056
 * bytes, lib/nghttp2_hd_huffman_data.c:29-94), dec_out receives
 * huff_decode_table (257 x 16 x {u16 fstate, u8 flags, u8 sym} = 16448 bytes,
 * :96-4980).  Either pointer may be NULL.  Returns 0. */
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_huff_tables(void *sym_out, void *dec_out);

/* ------------------------------------------------------------------ */
/* Sizing helpers (host-only, no GPU needed)                           */
/* ------------------------------------------------------------------ */

/* Upper bound of the encoded pool for `raw_bytes` bytes in `n` strings:
 * every symbol is at most 30 bits (RFC 7541 App. B), plus one padding byte
 * per string, rounded up to 16. */
NGHTTP2_AMD_EXTERN size_t nghttp2_amd_hd_huff_encode_bound(uint64_t raw_bytes, uint32_t n);

/* Size of the decode output pool nghttp2_amd_hd_huff_decode_batch_auto needs
 * for an encoded pool of `enc_bytes` bytes in `n` strings:
 * floor(8 * enc_bytes / 5) + 4 * n, rounded up. */
NGHTTP2_AMD_EXTERN size_t nghttp2_amd_hd_huff_decode_bound(uint64_t enc_bytes, uint32_t n);

/* Bytes of device workspace nghttp2_amd_hd_huff_encode_batch and
 * nghttp2_amd_hd_huff_decode_slots need for `n` strings. */
NGHTTP2_AMD_EXTERN size_t nghttp2_amd_hd_huff_workspace_size(uint32_t n);

/* A workspace size for nghttp2_amd_hd_huff_encode_batch that is also valid
 * for earlier versions of the library, which kept per-piece bit counts for
 * `raw_bytes` raw bytes in `n` strings.  Any size >=
 * nghttp2_amd_hd_huff_workspace_size(n) is valid; the current kernels use
 * only that much. */
NGHTTP2_AMD_EXTERN size_t nghttp2_amd_hd_huff_encode_workspace_size(uint64_t raw_bytes, uint32_t n);

/* ------------------------------------------------------------------ */
/* Batched device-resident API                                          */
/* ------------------------------------------------------------------ */

/*
 * Encode N strings.  Replaces, for a whole batch, emit_string's
 * nghttp2_hd_huff_encode_count + nghttp2_hd_huff_encode pair
 * (lib/nghttp2_hd.c:1009, :1037; lib/nghttp2_hd_huffman.c:34-104).
 *
 *   src, src_off[n+1] : raw strings (device)
 *   dst               : encoded pool (device), >= dst_cap bytes
 *   dst_off[n+1]      : OUT: encoded string i = dst[dst_off[i]..dst_off[i+1]);
 *                       dst_off[i+1]-dst_off[i] == nghttp2_hd_huff_encode_count
 *   workspace         : device scratch, >= nghttp2_amd_hd_huff_workspace_size(n)
 *
 * Output bytes equal lib/nghttp2_hd_huffman.c's, including the EOS-prefix
 * (all ones) padding of the last byte.  Size dst_cap by
 * nghttp2_amd_hd_huff_encode_bound(src_off[n]-src_off[0], n); the kernels
 * never write past dst_cap.  Offsets are uint32: when the encoded total
 * would pass min(dst_cap, 0xFFFFFFFE), dst_off[n] = NGHTTP2_AMD_OFF_OVERFLOW
 * (check it after the stream synchronises) and the batch must be split: the
 * tiles of 256 strings that fit may already be written, nothing at or past
 * dst_cap is, and no offset of the batch is valid.  A batch holding a
 * string longer than NGHTTP2_AMD_ENCODE_MAX_STRING raw bytes (its code bits
 * would not fit the kernels' 32-bit counts), or a tile of 256 consecutive
 * strings (256 k .. 256 k + 255) whose encoded output may reach
 * NGHTTP2_AMD_ENCODE_MAX_TILE bytes (a wave places its output bits in 32-bit
 * positions), is marked the same way.  The tile test is conservative: it
 * sums each string's output rounded down to 64 KiB units and marks the tile
 * when that sum comes within 256 units of 2^13 (2^29 bytes), so a tile whose
 * output is between 2^29 - 16 MiB and 2^29 bytes may be marked too.  Header
 * strings are far below both (nghttp2 caps a field at 64 KiB,
 * NGHTTP2_HD_MAX_NV).
 */
#define NGHTTP2_AMD_ENCODE_MAX_STRING (0xFFFFFFFFu / 30u)
#define NGHTTP2_AMD_ENCODE_MAX_TILE (1u << 29)
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_huff_encode_batch(const uint8_t *src, const uint32_t *src_off,
                                     uint32_t n, uint8_t *dst, size_t dst_cap,
                                     uint32_t *dst_off, void *workspace,
                                     size_t workspace_size, void *stream);

/*
 * HPACK string literals, batched: emit_string (lib/nghttp2_hd.c:1001-1044)
 * for N strings.  Literal i = dst[dst_off[i]..dst_off[i+1]) is
 *   H | length    the H bit (0x80) iff the Huffman form is strictly shorter
 *                 than the raw string (:1011), and the payload length as a
 *                 7-bit-prefix integer (count_encoded_length / encode_length,
 *                 :823-863, RFC 7541 5.1);
 *   payload       the Huffman bytes (nghttp2_hd_huff_encode) or the raw ones.
 * The literals are back to back in string order, ready to be spliced into
 * header blocks in wire order.  Two launches: the encode count (code bits
 * per string, tile sums of the literal lengths) and the encode pack, which
 * writes every literal -- prefix and payload -- straight into dst (no
 * intermediate Huffman pool); a batch of at most 256 strings takes one
 * launch that does both (the workspace is then not touched).
 *
 *   raw_bytes : src_off[n] - src_off[0] (sizes the bounds below)
 *   dst_cap   : >= nghttp2_amd_hd_emit_strings_bound(raw_bytes, n)
 *   workspace : device scratch (the tile sums),
 *               >= nghttp2_amd_hd_emit_strings_workspace_size(raw_bytes, n)
 */
NGHTTP2_AMD_EXTERN size_t nghttp2_amd_hd_emit_strings_bound(uint64_t raw_bytes, uint32_t n);
NGHTTP2_AMD_EXTERN size_t nghttp2_amd_hd_emit_strings_workspace_size(uint64_t raw_bytes, uint32_t n);
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_emit_strings_batch(const uint8_t *src, const uint32_t *src_off,
                                      uint32_t n, uint64_t raw_bytes, uint8_t *dst,
                                      size_t dst_cap, uint32_t *dst_off, void *workspace,
                                      size_t workspace_size, void *stream);

/*
 * Encoded lengths only: enc_len[i] = nghttp2_hd_huff_encode_count(string i)
 * (lib/nghttp2_hd_huffman.c:34-43).
 */
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_huff_encode_count_batch(const uint8_t *src,
                                           const uint32_t *src_off, uint32_t n,
                                           uint32_t *enc_len, void *stream);

/*
 * Output slots for a decode batch: dst_off[i+1]-dst_off[i] =
 * floor(8*E_i/5)+1, the reference's allocation for a Huffman literal
 * (nghttp2_huff_estimate_decode_length, lib/nghttp2_hd_huffman.h:76-78,
 * used at lib/nghttp2_hd.c:2080-2082 / :2166-2168).  dst_off[n] is the
 * pool size to allocate.
 */
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_huff_decode_slots(const uint32_t *src_off, uint32_t n,
                                     uint32_t *dst_off, void *workspace,
                                     size_t workspace_size, void *stream);

/*
 * Decode N whole Huffman strings (each call is final, fin=1).  Replaces,
 * for a batch, hd_inflate_read_huff's nghttp2_hd_huff_decode_context_init +
 * nghttp2_hd_huff_decode(..., fin=1) + nghttp2_hd_huff_decode_failure_state
 * (lib/nghttp2_hd.c:1728-1751, :2076, :2162;
 * lib/nghttp2_hd_huffman.c:106-147).
 *
 *   src, src_off[n+1] : encoded strings (device)
 *   dst, dst_off[n+1] : output slots (device); string i's decoded bytes are
 *                       written to dst[dst_off[i] ...]
 *   status[n]         : OUT: decoded length (>= 0), or
 *                       NGHTTP2_AMD_ERR_HEADER_COMP (-523) exactly when the
 *                       reference returns it (non-accepting end state,
 *                       including EOS decoded), or
 *                       NGHTTP2_AMD_ERR_BUFFER_ERROR (-502) when the slot is
 *                       smaller than the decoded length.
 *   fstate[n], flags[n] : OUT, optional (NULL to skip): the final
 *                       nghttp2_hd_huff_decode_context {fstate, flags}
 *                       (lib/nghttp2_hd_huffman.h:56-60) after the string;
 *                       fstate == 0x100 <=> failure_state().
 *
 * On -523 the bytes decoded before the failure are still written (as the
 * reference leaves them in buf), so dst matches the reference byte for byte.
 */
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_huff_decode_batch(const uint8_t *src, const uint32_t *src_off,
                                     uint32_t n, uint8_t *dst,
                                     const uint32_t *dst_off, int32_t *status,
                                     uint16_t *fstate, uint8_t *flags,
                                     void *stream);

/*
 * Same as nghttp2_amd_hd_huff_decode_batch, with the engine placing the
 * output in the same launch, densely: the batch is cut into tasks of 64
 * consecutive strings (t0 = 64 k), a task possibly split into two tasks of
 * 32 (t0 = 64 k, 64 k + 32: the engine splits the last tasks of each
 * workgroup's share so that its waves finish together), and the strings of
 * each task are back to back from the task's base
 *   base(t0) = 4 * (ceil(floor(8 x_t0 / 5) / 4) + t0),  x_t0 = src_off[t0] - src_off[0],
 * so dst_off[i] (OUT, n+1 entries) = base(t0) + the decoded bytes of the
 * task's strings before i, and dst_off[n] = the end of the last string
 * (dst_off is authoritative; which tasks were split is not specified).
 * Every string keeps the reference's allocation inside its task's span
 * (base(t1) - base(t0) >= the sum of floor(8 E_i / 5) + 1 over the task
 * [t0, t1)), so no
 * string can overflow; bytes between the end of a task's output and the
 * next task's base are unspecified.  dst (16-byte aligned) must hold
 * nghttp2_amd_hd_huff_decode_bound(E_total, n) bytes.  String i gets -502
 * when 4 * (ceil(floor(8 x_{i+1} / 5) / 4) + i + 1) > dst_cap (a pool
 * smaller than the bound); no byte at or past dst_cap is written and dst_off
 * entries saturate at dst_cap.  src_off must be non-decreasing: a task
 * holding a descending pair reports NGHTTP2_AMD_ERR_INVALID_ARGUMENT for its
 * strings and writes nothing for them.  Offsets
 * are uint32: dst_cap > 0xFFFFFFFF returns NGHTTP2_AMD_ERR_INVALID_ARGUMENT
 * (split a batch whose decode_bound passes 4 GiB).
 *
 * enc_bytes is the batch's encoded size, src_off[n] - src_off[0] (the value
 * that sized dst by nghttp2_amd_hd_huff_decode_bound).  It only picks the
 * kernel instance: a mean of at most 48 bytes per string (header-sized
 * strings) decodes whole strings as 64-byte items, a larger one cuts strings
 * into 40-byte pieces.  Both are exact for any input, so a wrong value costs
 * time, never correctness.  dst_cap does not enter the pick.
 */
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_huff_decode_batch_auto(const uint8_t *src, const uint32_t *src_off,
                                          uint32_t n, uint64_t enc_bytes, uint8_t *dst,
                                          size_t dst_cap, uint32_t *dst_off, int32_t *status,
                                          uint16_t *fstate, uint8_t *flags, void *stream);

/*
 * The reference's nibble-stepped FSM itself (lib/nghttp2_hd_huffman.c:111-143
 * over huff_decode_table, :122-133), batched: an exact cross-check of the
 * canonical decoder and the path for chunked (streaming) input.  Each string
 * i starts from the decode context {init_fstate[i], init_flags[i]} (both
 * NULL: nghttp2_hd_huff_decode_context_init, :106-109), the final context is
 * written to fstate/flags (optional), and `final` is the reference's fin
 * flag: when nonzero a non-accepting end state gives -523, else status is
 * the number of bytes written (the reference returns srclen then; the
 * caller checks fstate == 0x100 for failure_state, :145-147).
 */
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_huff_decode_fsm_batch(const uint8_t *src, const uint32_t *src_off,
                                         uint32_t n, uint8_t *dst, const uint32_t *dst_off,
                                         int32_t *status, uint16_t *fstate, uint8_t *flags,
                                         const uint16_t *init_fstate,
                                         const uint8_t *init_flags, int final,
                                         void *stream);

/* ------------------------------------------------------------------ */
/* Header-name tokens and name hash              */
/* ------------------------------------------------------------------ */
/*
 * Replaces lookup_token (lib/nghttp2_hd.c:137-520) and name_hash
 * (lib/nghttp2_hd.c:536-547), both static in the reference and called per
 * header field by deflate_nv (:1388-1393) and the inflater (:1811).
 *
 * nghttp2_amd_hd_name_tokens_batch: N names in the batch layout (device pool
 * + uint32 offsets[N+1], pool readable to align_up(off[N], 16) + 16);
 * token[i] = lookup_token(name i) (-1, or NGHTTP2_TOKEN_* of
 * lib/nghttp2_hd.h:56-116: the first static-table index of a static name,
 * 61..67 for te, connection, keep-alive, proxy-connection, upgrade,
 * :protocol, priority); hash[i] = 32-bit FNV-1a of name i (equal to the
 * reference's static_table[token].hash for a static name).  Device pointers,
 * asynchronous on `stream`.
 *
 * nghttp2_amd_hd_lookup_token / nghttp2_amd_hd_name_hash: the same for one
 * host name (what a single deflate_nv call binds).
 */
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_name_tokens_batch(const uint8_t *names,
                                                        const uint32_t *name_off, uint32_t n,
                                                        int32_t *token, uint32_t *hash,
                                                        void *stream);
NGHTTP2_AMD_EXTERN int32_t nghttp2_amd_hd_lookup_token(const uint8_t *name, size_t namelen);
NGHTTP2_AMD_EXTERN uint32_t nghttp2_amd_hd_name_hash(const uint8_t *name, size_t namelen);

/* ------------------------------------------------------------------ */
/* Batched HPACK inflate front-end               */
/* ------------------------------------------------------------------ */
/*
 * An inflater is one connection's HPACK decoding context (dynamic table,
 * table size settings), as nghttp2_hd_inflater (lib/nghttp2_hd.h).
 * nghttp2_amd_hd_inflate_blocks decodes a batch of complete header blocks,
 * block i against inflaters[i] (blocks of one connection in order), with
 * every Huffman literal of the batch decoded in ONE GPU call.  Per block it
 * behaves as nghttp2_hd_inflate_hd3 (nghttp2.h:6623) called with in_final=1
 * until NGHTTP2_HD_INFLATE_FINAL, then nghttp2_hd_inflate_end_headers
 * (nghttp2.h:6636): the same fields, the same dynamic table evolution, the
 * same errors (NGHTTP2_ERR_HEADER_COMP, sticky per inflater).
 */
typedef struct nghttp2_amd_hd_inflater nghttp2_amd_hd_inflater;

/* One emitted header field: name and value are NUL-terminated byte strings
 * in the caller's arena; flags = NGHTTP2_NV_FLAG_NO_INDEX (1) for a
 * never-indexed literal (nghttp2.h:574-613). */
typedef struct {
  uint32_t block;
  uint32_t name_off, name_len;
  uint32_t value_off, value_len;
  uint8_t flags;
} nghttp2_amd_hd_nv;

/* nghttp2_hd_inflate_new (nghttp2.h:6277): dynamic table of 4096 bytes. */
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_inflate_new(nghttp2_amd_hd_inflater **inflater_ptr);
/* nghttp2_hd_inflate_del (nghttp2.h:6302) */
NGHTTP2_AMD_EXTERN void nghttp2_amd_hd_inflate_del(nghttp2_amd_hd_inflater *inflater);
/* nghttp2_hd_inflate_change_table_size (nghttp2.h:6331): a smaller value
 * than the current maximum requires a size update at the head of the next
 * block. */
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_inflate_change_table_size(nghttp2_amd_hd_inflater *inflater,
                                             size_t settings_max_dynamic_table_size);
/* nghttp2_hd_inflate_get_num_table_entries / get_table_entry /
 * get_dynamic_table_size / get_max_dynamic_table_size (nghttp2.h:6646-6678);
 * idx is 1-based over static + dynamic table. */
NGHTTP2_AMD_EXTERN size_t nghttp2_amd_hd_inflate_get_num_table_entries(nghttp2_amd_hd_inflater *inflater);
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_inflate_get_table_entry(nghttp2_amd_hd_inflater *inflater,
                                           size_t idx, const uint8_t **name, size_t *namelen,
                                           const uint8_t **value, size_t *valuelen);
NGHTTP2_AMD_EXTERN size_t nghttp2_amd_hd_inflate_get_dynamic_table_size(nghttp2_amd_hd_inflater *inflater);
NGHTTP2_AMD_EXTERN size_t nghttp2_amd_hd_inflate_get_max_dynamic_table_size(nghttp2_amd_hd_inflater *inflater);

/*
 * Inflate nblocks complete header blocks (host memory).  Fields go to
 * nva[0..*nva_used) in block order, their bytes to arena[0..*arena_used).
 * block_status[i] = fields of block i, or NGHTTP2_AMD_ERR_HEADER_COMP (the
 * fields before the error stay emitted, as the reference emits them one at
 * a time; the inflater turns bad), or NGHTTP2_AMD_ERR_BUFFER_ERROR when
 * nva / arena ran out (that block and the rest are not applied).  The GPU
 * work is asynchronous on `stream` and synchronised before return; a batch
 * without Huffman literals makes no GPU call.  The library keeps one
 * process-wide engine (pinned and device buffers, parse state) for this
 * call, so concurrent calls are serialised whole, host passes included; the
 * engine keeps its per-block buffers across calls and releases the surplus
 * when a call is far smaller than an earlier one.
 */
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_inflate_blocks(nghttp2_amd_hd_inflater *const *inflaters,
                                  uint32_t nblocks, const uint8_t *const *blocks,
                                  const size_t *block_lens, nghttp2_amd_hd_nv *nva,
                                  size_t nva_cap, size_t *nva_used, uint8_t *arena,
                                  size_t arena_cap, size_t *arena_used, int32_t *block_status,
                                  void *stream);

/* ------------------------------------------------------------------ */
/* Batched HPACK deflate front-end                                      */
/* ------------------------------------------------------------------ */
/*
 * A deflater is one connection's HPACK encoding context (nghttp2_hd_deflater,
 * lib/nghttp2_hd.h).  nghttp2_amd_hd_deflate_blocks encodes a batch of
 * header lists, list i with deflaters[i] (lists of one connection in
 * order); every string literal of the batch is framed by ONE GPU call
 * (nghttp2_amd_hd_emit_strings_batch).  Block i's wire is byte-identical to
 * nghttp2_hd_deflate_hd2 (nghttp2.h:6127) on the same deflater state:
 * the same table size updates, table search, indexing decisions (never
 * index authorization, cookies shorter than 20 bytes and NO_INDEX fields;
 * no indexing for :path, age, content-length, etag, if-modified-since,
 * if-none-match, location, set-cookie and entries over 3/4 of the table)
 * and the same Huffman-or-raw literals.
 */
typedef struct nghttp2_amd_hd_deflater nghttp2_amd_hd_deflater;

/* Same layout as nghttp2_nv (nghttp2.h:574-613); flags bit 0 =
 * NGHTTP2_NV_FLAG_NO_INDEX. */
typedef struct {
  const uint8_t *name;
  const uint8_t *value;
  size_t namelen;
  size_t valuelen;
  uint8_t flags;
} nghttp2_amd_nv;

/* nghttp2_hd_deflate_new (nghttp2.h:6003) */
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_deflate_new(nghttp2_amd_hd_deflater **deflater_ptr,
                               size_t max_deflate_dynamic_table_size);
/* nghttp2_hd_deflate_del (nghttp2.h:6031) */
NGHTTP2_AMD_EXTERN void nghttp2_amd_hd_deflate_del(nghttp2_amd_hd_deflater *deflater);
/* nghttp2_hd_deflate_change_table_size (nghttp2.h:6057) */
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_deflate_change_table_size(nghttp2_amd_hd_deflater *deflater,
                                             size_t settings_max_dynamic_table_size);
/* nghttp2_hd_deflate_get_num_table_entries / get_table_entry /
 * get_dynamic_table_size (nghttp2.h:6221-6253); idx is 1-based. */
NGHTTP2_AMD_EXTERN size_t nghttp2_amd_hd_deflate_get_num_table_entries(nghttp2_amd_hd_deflater *deflater);
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_deflate_get_table_entry(nghttp2_amd_hd_deflater *deflater,
                                           size_t idx, const uint8_t **name, size_t *namelen,
                                           const uint8_t **value, size_t *valuelen);
NGHTTP2_AMD_EXTERN size_t nghttp2_amd_hd_deflate_get_dynamic_table_size(nghttp2_amd_hd_deflater *deflater);
/* nghttp2_hd_deflate_get_max_dynamic_table_size (nghttp2.h:6253) */
NGHTTP2_AMD_EXTERN size_t nghttp2_amd_hd_deflate_get_max_dynamic_table_size(nghttp2_amd_hd_deflater *deflater);
/* nghttp2_hd_deflate_bound (nghttp2.h:6209): an upper bound of one list's
 * wire; the sum over a batch bounds out_cap. */
NGHTTP2_AMD_EXTERN size_t nghttp2_amd_hd_deflate_bound(nghttp2_amd_hd_deflater *deflater,
                                    const nghttp2_amd_nv *nva, size_t nvlen);

/*
 * Deflate nblocks header lists (host memory): list i is
 * nva[block_nv_off[i]..block_nv_off[i+1]).  Block i's wire is
 * out[out_off[i]..out_off[i+1]); block_status[i] = its length, or
 * NGHTTP2_AMD_ERR_HEADER_COMP for a deflater already bad, or
 * NGHTTP2_AMD_ERR_BUFFER_ERROR when out_cap ran out (the deflater turns bad,
 * as nghttp2_hd_deflate_hd2's INSUFF_BUFSIZE does).  The GPU work is
 * asynchronous on `stream` and synchronised before return.
 */
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_deflate_blocks(nghttp2_amd_hd_deflater *const *deflaters,
                                  uint32_t nblocks, const nghttp2_amd_nv *nva,
                                  const uint32_t *block_nv_off, uint8_t *out, size_t out_cap,
                                  uint32_t *out_off, int32_t *block_status, void *stream);

/*
 * One header list into a caller buffer, as nghttp2_hd_deflate_hd2
 * (nghttp2.h:6127; lib/nghttp2_hd.c:1525-1555): the wire length, or
 * NGHTTP2_AMD_ERR_INSUFF_BUFSIZE when buflen is too small (the deflater
 * turns bad, as the reference's does), or NGHTTP2_AMD_ERR_HEADER_COMP for a
 * deflater already bad.  A batch of one list on nghttp2_amd_hd_deflate_blocks
 * (its literals framed by the GPU); host buffers, synchronous.
 */
NGHTTP2_AMD_EXTERN ptrdiff_t nghttp2_amd_hd_deflate_hd2(nghttp2_amd_hd_deflater *deflater,
                                                         uint8_t *buf, size_t buflen,
                                                         const nghttp2_amd_nv *nva, size_t nvlen,
                                                         void *stream);

/* Same layout as nghttp2_vec (nghttp2.h:5910-5919). */
typedef struct {
  uint8_t *base;
  size_t len;
} nghttp2_amd_vec;

/*
 * nghttp2_hd_deflate_hd_vec2 (nghttp2.h:6179; lib/nghttp2_hd.c:1563-1594):
 * as nghttp2_amd_hd_deflate_hd2, the wire written across the chunks
 * vec[0..veclen) in order (each filled before the next); INSUFF_BUFSIZE when
 * their total is too small, including veclen == 0 and zero-length chunks.
 * On INSUFF_BUFSIZE with several chunks, none of them is written (the
 * reference leaves the bytes it had written before it ran out).
 */
NGHTTP2_AMD_EXTERN ptrdiff_t nghttp2_amd_hd_deflate_hd_vec2(nghttp2_amd_hd_deflater *deflater,
                                                             const nghttp2_amd_vec *vec,
                                                             size_t veclen,
                                                             const nghttp2_amd_nv *nva,
                                                             size_t nvlen, void *stream);

/*
 * The HPACK prefix-integer decoder the inflate front-end parses with, as
 * nghttp2_hd_decode_length (lib/nghttp2_hd.h:416-419; lib/nghttp2_hd.c:
 * 882-945), resumable byte by byte: decode from in[0..last - in) with a
 * `prefix`-bit first byte, continuing a previous call's partial value
 * `initial` at `shift` (both 0 at the start of an integer).  Returns the
 * bytes consumed, or -1 on overflow past UINT32_MAX (a shift of 32 bits or
 * more included); *fin = 1 once the integer is complete (*res its value),
 * else *res and *shift_ptr carry the partial state to the next call.
 * Host-only.
 */
NGHTTP2_AMD_EXTERN ptrdiff_t nghttp2_amd_hd_decode_length(uint32_t *res, size_t *shift_ptr, int *fin,
                                                           uint32_t initial, size_t shift,
                                                           const uint8_t *in, const uint8_t *last,
                                                           size_t prefix);

/* ------------------------------------------------------------------ */
/* One batch over several GPUs                       */
/* ------------------------------------------------------------------ */
/*
 * Strings are independent, so a batch shards into contiguous string ranges
 * balanced by bytes, one per device, with no exchange between devices (no
 * RCCL, xGMI unused).  A sharded engine owns one host worker thread, one HIP
 * stream and its own device buffers per entry of its device list (a device
 * may repeat: several shards on one GPU); the table of each kernel is staged
 * per device.  This is nghttp2's concurrency model (one session per thread,
 * nothing shared; doc/programmers-guide.rst:35-40) with a GPU behind each
 * thread.  A sharded engine is used by one caller thread at a time; distinct
 * engines may run concurrently.
 *
 * The shard outputs are merged into one batch: shard k's output bytes follow
 * shard k-1's, and its offsets are rebased by the bytes before it.  Encode:
 * the result equals nghttp2_amd_hd_huff_encode_batch of the whole batch.
 * Decode: each shard is laid out as nghttp2_amd_hd_huff_decode_batch_auto
 * lays out a batch of its strings (dense per task, counted from the shard's
 * first string), shifted by the bytes of the shards before it; dst_off,
 * status, fstate and flags are per string as for the unsharded call.
 */
typedef struct nghttp2_amd_hd_sharded nghttp2_amd_hd_sharded;

/* Byte-balanced contiguous cut of a batch of n strings (offsets off[n+1])
 * into nshards ranges: cuts[0] = 0, cuts[nshards] = n, shard k holds the
 * strings [cuts[k], cuts[k+1]), which start at or after its 1/nshards share
 * of the bytes.  Host-only.  Returns 0 or NGHTTP2_AMD_ERR_INVALID_ARGUMENT. */
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_shard_bounds(const uint32_t *off, uint32_t n, uint32_t nshards,
                                                   uint32_t *cuts);

/* A sharded engine over ndevices HIP device ids (repeats allowed).  Returns
 * 0, NGHTTP2_AMD_ERR_INVALID_ARGUMENT (no device, an id out of range) or
 * NGHTTP2_AMD_ERR_FATAL / _NOMEM (a stream or thread could not be made). */
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_sharded_new(nghttp2_amd_hd_sharded **out, const int *devices,
                                                  uint32_t ndevices);
NGHTTP2_AMD_EXTERN void nghttp2_amd_hd_sharded_del(nghttp2_amd_hd_sharded *s);
NGHTTP2_AMD_EXTERN uint32_t nghttp2_amd_hd_sharded_count(const nghttp2_amd_hd_sharded *s);

/*
 * Host-resident batch (pinned memory gives the full PCIe rate; pageable
 * memory works and copies through the runtime's staging).  src must be
 * readable to align_up(src_off[n], 16) + 16 (the pool padding of every batch
 * call).  Each shard: H2D of its bytes and offsets, the engine kernels, D2H
 * of its output straight to its merged position.  Synchronous: returns when
 * every shard's output is in dst.
 *
 * encode: Huffman encode; dst_off[n+1] merged (dst_off[0] = 0).  When the
 *   merged output passes dst_cap or the uint32 offsets, nothing is written to
 *   dst, dst_off[n] = NGHTTP2_AMD_OFF_OVERFLOW and the call returns
 *   NGHTTP2_AMD_ERR_BUFFER_ERROR (split the batch).
 * decode: decode with final=1 (status per string as decode_batch_auto);
 *   dst_cap >= nghttp2_amd_hd_huff_decode_bound(E, n) + 32 * shards always
 *   suffices (E = src_off[n] - src_off[0]); a smaller pool that the merged
 *   output does not fit returns NGHTTP2_AMD_ERR_BUFFER_ERROR with nothing
 *   written to dst.  fstate and flags may both be NULL.
 */
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_sharded_encode(nghttp2_amd_hd_sharded *s, const uint8_t *src,
                                                     const uint32_t *src_off, uint32_t n, uint8_t *dst,
                                                     size_t dst_cap, uint32_t *dst_off);
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_sharded_decode(nghttp2_amd_hd_sharded *s, const uint8_t *src,
                                                     const uint32_t *src_off, uint32_t n, uint8_t *dst,
                                                     size_t dst_cap, uint32_t *dst_off, int32_t *status,
                                                     uint16_t *fstate, uint8_t *flags);

/*
 * Device-resident shards: shards[k] lives on the engine's k-th device (cut
 * by the caller, e.g. with nghttp2_amd_hd_shard_bounds; its src_off may be
 * absolute or rebased -- the engine calls take them as given).  Each shard
 * runs nghttp2_amd_hd_huff_encode_batch / _decode_batch_auto on its device
 * and stream; its output stays there with shard-local offsets, and the
 * engine reports out_bytes (its dst_off[n]) and out_base (the bytes of the
 * shards before it, its position in the merged batch).  Synchronous.
 * Returns 0 or the first failing shard's error (each shard's own in rv).
 */
typedef struct {
  const uint8_t *src;        /* IN  pool on the shard's device (16-byte aligned, padded) */
  const uint32_t *src_off;   /* IN  offsets[n+1] on the shard's device */
  uint32_t n;                /* IN  strings of the shard */
  uint64_t in_bytes;         /* IN  decode: src_off[n] - src_off[0]; encode: raw bytes */
  uint8_t *dst;              /* IN  output pool on the shard's device */
  size_t dst_cap;            /* IN */
  uint32_t *dst_off;         /* IN  offsets[n+1] on the shard's device */
  int32_t *status;           /* IN  decode: status[n] on the device (encode: unused) */
  uint16_t *fstate;          /* IN  decode: optional (with flags) */
  uint8_t *flags;            /* IN  decode: optional (with fstate) */
  uint64_t out_bytes;        /* OUT the shard's output bytes (dst_off[n]) */
  uint64_t out_base;         /* OUT its first byte in the merged batch */
  int rv;                    /* OUT the shard's nghttp2_error (0) */
} nghttp2_amd_hd_shard;
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_sharded_encode_dev(nghttp2_amd_hd_sharded *s,
                                                         nghttp2_amd_hd_shard *shards);
NGHTTP2_AMD_EXTERN int nghttp2_amd_hd_sharded_decode_dev(nghttp2_amd_hd_sharded *s,
                                                         nghttp2_amd_hd_shard *shards);

#ifdef __cplusplus
}
#endif

#endif /* NGHTTP2_AMD_HD_H */
