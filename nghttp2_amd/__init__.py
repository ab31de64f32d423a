"""nghttp2_amd -- MI355X-native HPACK Huffman engine (host side).

The product is the HIP/C shared library nghttp2_amd/lib/libnghttp2_amd_hd.so
(sources in nghttp2_amd/csrc, C ABI in include/nghttp2_amd_hd.h).  This
package is the thin Python binding over that C ABI used by bench.py, the
batched drivers and the tests: torch is only the device-memory / stream
plumbing.  There is no CPU fallback: every compute call goes to the HIP
library and raises if it is missing.
"""
from .hd import (  # noqa: F401
    HpackDeflater,
    HpackInflater,
    HuffmanBatchCodec,
    NGHTTP2_ERR_BUFFER_ERROR,
    NGHTTP2_ERR_HEADER_COMP,
    NGHTTP2_ERR_INSUFF_BUFSIZE,
    NGHTTP2_ERR_INVALID_ARGUMENT,
    decode_length,
    lib,
    lib_path,
    deflate_blocks,
    inflate_blocks,
    tables_ref_layout,
)

__version__ = "0.1.0"
