"""oracle/hpack_oracle.py -- TEST INFRASTRUCTURE ONLY.

Pure-Python restatement of nghttp2's HPACK inflater, used as the parity
checker of the batched inflate front-end (nghttp2_amd_hd_inflate_blocks).
Nothing in the product imports it.  Huffman literals go through the C oracle
(oracle/huff_oracle.c, nghttp2_hd_huff_decode with fin=1).

Restates (citations are /root/reference paths):
  nghttp2_hd_inflate_hd_nv          lib/nghttp2_hd.c:1919-2281 (in_final=1)
  nghttp2_hd_inflate_end_headers    lib/nghttp2_hd.c:2283-2287
  nghttp2_hd_inflate_change_table_size  lib/nghttp2_hd.c:1290-1322
  decode_length                     lib/nghttp2_hd.c:882-945
  hd_inflate_commit_indexed/newname/indname  lib/nghttp2_hd.c:1780-1875
  add_hd_table_incremental          lib/nghttp2_hd.c:1130-1195
  static table                      RFC 7541 Appendix A
"""
from . import oracle as O

MAX_NV = 65536           # NGHTTP2_HD_MAX_NV
ENTRY_OVERHEAD = 32      # NGHTTP2_HD_ENTRY_OVERHEAD
DEFAULT_TABLE = 4096     # NGHTTP2_HD_DEFAULT_MAX_BUFFER_SIZE
HEADER_COMP = -523
NO_INDEX = 1             # NGHTTP2_NV_FLAG_NO_INDEX

STATIC = [
    (b":authority", b""), (b":method", b"GET"), (b":method", b"POST"), (b":path", b"/"),
    (b":path", b"/index.html"), (b":scheme", b"http"), (b":scheme", b"https"),
    (b":status", b"200"), (b":status", b"204"), (b":status", b"206"), (b":status", b"304"),
    (b":status", b"400"), (b":status", b"404"), (b":status", b"500"),
    (b"accept-charset", b""), (b"accept-encoding", b"gzip, deflate"),
    (b"accept-language", b""), (b"accept-ranges", b""), (b"accept", b""),
    (b"access-control-allow-origin", b""), (b"age", b""), (b"allow", b""),
    (b"authorization", b""), (b"cache-control", b""), (b"content-disposition", b""),
    (b"content-encoding", b""), (b"content-language", b""), (b"content-length", b""),
    (b"content-location", b""), (b"content-range", b""), (b"content-type", b""),
    (b"cookie", b""), (b"date", b""), (b"etag", b""), (b"expect", b""), (b"expires", b""),
    (b"from", b""), (b"host", b""), (b"if-match", b""), (b"if-modified-since", b""),
    (b"if-none-match", b""), (b"if-range", b""), (b"if-unmodified-since", b""),
    (b"last-modified", b""), (b"link", b""), (b"location", b""), (b"max-forwards", b""),
    (b"proxy-authenticate", b""), (b"proxy-authorization", b""), (b"range", b""),
    (b"referer", b""), (b"refresh", b""), (b"retry-after", b""), (b"server", b""),
    (b"set-cookie", b""), (b"strict-transport-security", b""), (b"transfer-encoding", b""),
    (b"user-agent", b""), (b"vary", b""), (b"via", b""), (b"www-authenticate", b"")]
assert len(STATIC) == 61


class _Fail(Exception):
    pass


class Inflater:
    def __init__(self):
        self.table = []                  # [0] = most recent
        self.size = 0
        self.max = DEFAULT_TABLE         # ctx.hd_table_bufsize_max
        self.settings_max = DEFAULT_TABLE
        self.min_max = 0xFFFFFFFF
        self.expect_size = False
        self.bad = False

    # lib/nghttp2_hd.c:1290-1322
    def change_table_size(self, v):
        self.settings_max = v
        if self.max > v:
            self.expect_size = True
            self.min_max = v
            self.max = v
            self._shrink()

    def _shrink(self):
        while self.size > self.max and self.table:
            n, v = self.table.pop()
            self.size -= len(n) + len(v) + ENTRY_OVERHEAD

    # add_hd_table_incremental, lib/nghttp2_hd.c:1130-1195
    def _add(self, n, v):
        room = len(n) + len(v) + ENTRY_OVERHEAD
        while self.size + room > self.max and self.table:
            a, b = self.table.pop()
            self.size -= len(a) + len(b) + ENTRY_OVERHEAD
        if room > self.max:
            return
        self.table.insert(0, (n, v))
        self.size += room

    def _get(self, idx):
        return STATIC[idx] if idx < 61 else self.table[idx - 61]

    def inflate_block(self, block):
        """One complete block (in_final=1, then end_headers).  Returns
        (status, fields): status = number of fields or HEADER_COMP; fields
        emitted before an error are returned too (the reference emits them
        one at a time)."""
        fields = []
        if self.bad:
            return HEADER_COMP, fields
        try:
            self._inflate(bytes(block), fields)
        except _Fail:
            self.bad = True
            return HEADER_COMP, fields
        return len(fields), fields

    def _inflate(self, b, fields):
        pos = [0]
        head = True

        # decode_length, lib/nghttp2_hd.c:882-945 (with in_final)
        def read_int(prefix, maxlen):
            if pos[0] >= len(b):
                raise _Fail()
            k = (1 << prefix) - 1
            n = b[pos[0]] & k
            pos[0] += 1
            if n == k:
                shift = 0
                while True:
                    if pos[0] >= len(b):
                        raise _Fail()
                    c = b[pos[0]]
                    pos[0] += 1
                    add = c & 0x7F
                    if shift >= 32 or (0xFFFFFFFF >> shift) < add:
                        raise _Fail()
                    add <<= shift
                    if 0xFFFFFFFF - add < n:
                        raise _Fail()
                    n += add
                    if not c & 0x80:
                        break
                    shift += 7
            if n > maxlen:
                raise _Fail()
            return n

        def read_str():
            if pos[0] >= len(b):
                raise _Fail()
            huff = b[pos[0]] & 0x80
            n = read_int(7, MAX_NV)
            if len(b) - pos[0] < n:
                raise _Fail()
            s = b[pos[0]:pos[0] + n]
            pos[0] += n
            if huff:
                rv, out, ctx = O.decode(s, final=1)
                if rv < 0 or O.failure_state(ctx):
                    raise _Fail()
                return out
            return s

        while pos[0] < len(b):
            c = b[pos[0]]
            if self.expect_size and (c & 0xE0) != 0x20:
                raise _Fail()
            if (c & 0xE0) == 0x20:
                if not head:
                    raise _Fail()
                v = read_int(5, min(self.min_max, self.settings_max))
                self.min_max = 0xFFFFFFFF
                self.expect_size = False
                self.max = v
                self._shrink()
                continue
            head = False
            if c & 0x80:
                idx = read_int(7, len(self.table) + 61)
                if idx == 0:
                    raise _Fail()
                n, v = self._get(idx - 1)
                fields.append((n, v, 0))
                continue
            index_required = bool(c & 0x40)
            no_index = (c & 0xF0) == 0x10
            if c in (0x40, 0x00, 0x10):
                pos[0] += 1
                name = read_str()
            else:
                idx = read_int(6 if index_required else 4, len(self.table) + 61)
                if idx == 0:
                    raise _Fail()
                name = self._get(idx - 1)[0]
            value = read_str()
            if index_required:
                self._add(name, value)
            fields.append((name, value, NO_INDEX if no_index else 0))
        if self.expect_size:  # the block ended in EXPECT_TABLE_SIZE (:2259-2266)
            raise _Fail()


def block_has_huffman(b):
    """Whether a complete block carries a Huffman string literal (the H bit of
    any literal): the wire is self-delimiting, so this is a stateless scan of
    the representations (lib/nghttp2_hd.c:1919-2288's opcode and literal
    framing).  Test infrastructure: which product cases need the GPU."""
    b = bytes(b)
    pos = 0

    def skip_int(prefix):
        nonlocal pos
        k = (1 << prefix) - 1
        n = b[pos] & k
        pos += 1
        if n == k:
            shift = 0
            while True:
                c = b[pos]
                pos += 1
                n += (c & 0x7F) << shift
                shift += 7
                if not c & 0x80:
                    break
        return n

    def lit():
        nonlocal pos
        h = b[pos] & 0x80
        n = skip_int(7)
        pos += n
        return bool(h)

    found = False
    while pos < len(b):
        c = b[pos]
        if (c & 0xE0) == 0x20:
            skip_int(5)
        elif c & 0x80:
            skip_int(7)
        else:
            if c in (0x40, 0x00, 0x10):
                pos += 1
                found |= lit()
            else:
                skip_int(6 if c & 0x40 else 4)
            found |= lit()
    return found


# ---------------------------------------------------------------------------
# Deflater (nghttp2_hd_deflate_hd2 per block)
# ---------------------------------------------------------------------------
_NEVER, _WITHOUT, _WITH = 2, 1, 0
_NO_INDEXING_NAMES = {b":path", b"age", b"content-length", b"etag", b"if-modified-since",
                      b"if-none-match", b"location", b"set-cookie"}
_STATIC_TOKEN = {}
for _i, (_n, _v) in enumerate(STATIC):
    _STATIC_TOKEN.setdefault(_n, _i)


class Deflater:
    """Restates nghttp2_hd_deflate_init2 (lib/nghttp2_hd.c:730-752),
    nghttp2_hd_deflate_change_table_size (:1274-1288),
    nghttp2_hd_deflate_hd_bufs (:1469-1505), deflate_nv (:1373-1467),
    search_hd_table / search_static_table / hd_map_find (:1201-1249,
    :566-589), hd_deflate_decide_indexing (:1358-1371) and the emit_*
    helpers (:975-1128); string literals through the C oracle's emit_string."""

    def __init__(self, max_deflate=4096):
        self.table, self.size = [], 0
        self.deflate_max = max_deflate
        self.max = 4096
        self.notify = False
        self.min_max = 0xFFFFFFFF
        if max_deflate < 4096:
            self.notify, self.max = True, max_deflate

    def change_table_size(self, v):
        nxt = min(v, self.deflate_max)
        self.max = nxt
        self.min_max = min(self.min_max, nxt)
        self.notify = True
        while self.size > self.max and self.table:
            a, b = self.table.pop()
            self.size -= len(a) + len(b) + ENTRY_OVERHEAD

    def _add(self, n, v):
        room = len(n) + len(v) + ENTRY_OVERHEAD
        while self.size + room > self.max and self.table:
            a, b = self.table.pop()
            self.size -= len(a) + len(b) + ENTRY_OVERHEAD
        if room <= self.max:
            self.table.insert(0, (n, v))
            self.size += room

    def deflate_block(self, fields):
        out = bytearray()
        if self.notify:
            mn = self.min_max
            self.notify, self.min_max = False, 0xFFFFFFFF
            if self.max > mn:
                out += O.encode_length(mn, 5, 0x20)
            out += O.encode_length(self.max, 5, 0x20)
        for f in fields:
            n, v = bytes(f[0]), bytes(f[1])
            flags = f[2] if len(f) > 2 else 0
            token = _STATIC_TOKEN.get(n, -1)
            if n == b"authorization" or (n == b"cookie" and len(v) < 20) or flags & NO_INDEX:
                mode = _NEVER
            elif n in _NO_INDEXING_NAMES or len(n) + len(v) + ENTRY_OVERHEAD > self.max * 3 // 4:
                mode = _WITHOUT
            else:
                mode = _WITH
            idx, exact = -1, False
            for t, (a, b) in enumerate(self.table):
                if a != n:
                    continue
                if idx < 0:
                    idx = 61 + t
                    if mode == _NEVER:
                        break
                if b == v:
                    idx, exact = 61 + t, True
                    break
            if not exact and token >= 0:
                idx = token
                if mode != _NEVER:
                    s = token
                    while s < 61 and STATIC[s][0] == n:
                        if STATIC[s][1] == v:
                            idx, exact = s, True
                            break
                        s += 1
            if exact:
                out += O.encode_length(idx + 1, 7, 0x80)
                continue
            if mode == _WITH:
                self._add(n, v)
            first = (0x40, 0x00, 0x10)[mode]
            if idx < 0:
                out.append(first)
                out += O.emit_string(n)
            else:
                out += O.encode_length(idx + 1, 6 if mode == _WITH else 4, first)
            out += O.emit_string(v)
        return bytes(out)


# ---------------------------------------------------------------------------
# Header-name tokens and name hash
# ---------------------------------------------------------------------------
# lookup_token (lib/nghttp2_hd.c:137-520): a static-table name gives its first
# static index (the NGHTTP2_TOKEN_* values 0..60, lib/nghttp2_hd.h:57-108);
# seven more names get 61..67 in enum order (lib/nghttp2_hd.h:109-115).
_EXTRA_TOKENS = [b"te", b"connection", b"keep-alive", b"proxy-connection", b"upgrade",
                 b":protocol", b"priority"]
_TOKENS = dict(_STATIC_TOKEN)
for _k, _n in enumerate(_EXTRA_TOKENS):
    _TOKENS[_n] = 61 + _k


def lookup_token(name):
    """lib/nghttp2_hd.c:137-520 -- exact, case-sensitive name match."""
    return _TOKENS.get(bytes(name), -1)


def name_hash(name):
    """32-bit FNV-1a, lib/nghttp2_hd.c:536-547 (the shift-add form of
    h *= 16777619)."""
    h = 2166136261
    for c in bytes(name):
        h ^= c
        h = (h + (h << 1) + (h << 4) + (h << 7) + (h << 8) + (h << 24)) & 0xFFFFFFFF
    return h


def name_tokens(names):
    """(token[], hash[]) for a list of names: what
    nghttp2_amd_hd_name_tokens_batch returns."""
    return [lookup_token(n) for n in names], [name_hash(n) for n in names]


# ---------------------------------------------------------------------------
# The same inflater in C (oracle/hpack_inflate_oracle.c): checked against the
# Python Inflater above (tests/test_inflate_c_oracle.py) and timed as the
# inflate front-end's CPU baseline (tools/bench_rows.py).
# ---------------------------------------------------------------------------
def _clib():
    import ctypes
    L = O.lib()
    if not getattr(L, "_ohi_bound", False):
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        L.ohi_new.restype = vp
        L.ohi_del.argtypes = [vp]
        L.ohi_change_table_size.argtypes = [vp, sz]
        L.ohi_num_entries.restype = sz
        L.ohi_num_entries.argtypes = [vp]
        L.ohi_table_size.restype = sz
        L.ohi_table_size.argtypes = [vp]
        L.ohi_get_entry.argtypes = [vp, sz, ctypes.POINTER(vp), ctypes.POINTER(sz),
                                    ctypes.POINTER(vp), ctypes.POINTER(sz)]
        L.ohi_inflate_block.restype = ctypes.c_long
        L.ohi_inflate_block.argtypes = [vp, vp, sz, vp, sz, ctypes.POINTER(sz), vp, sz,
                                        ctypes.POINTER(sz)]
        L.ohi_inflate_batch_timed.restype = ctypes.c_double
        L.ohi_inflate_batch_timed.argtypes = [vp, vp, vp, ctypes.c_uint32, ctypes.c_uint32,
                                              ctypes.c_int, ctypes.POINTER(ctypes.c_long)]
        L._ohi_bound = True
    return L


class CInflater:
    """oracle/hpack_inflate_oracle.c behind the Inflater interface."""

    def __init__(self):
        self.L = _clib()
        self.p = self.L.ohi_new()
        assert self.p

    def __del__(self):
        if getattr(self, "p", None):
            self.L.ohi_del(self.p)
            self.p = None

    def change_table_size(self, v):
        self.L.ohi_change_table_size(self.p, v)

    @property
    def table(self):
        import ctypes
        out = []
        for k in range(self.L.ohi_num_entries(self.p)):
            n, v = ctypes.c_void_p(), ctypes.c_void_p()
            nl, vl = ctypes.c_size_t(), ctypes.c_size_t()
            self.L.ohi_get_entry(self.p, k, ctypes.byref(n), ctypes.byref(nl), ctypes.byref(v),
                                 ctypes.byref(vl))
            out.append((ctypes.string_at(n, nl.value) if nl.value else b"",
                        ctypes.string_at(v, vl.value) if vl.value else b""))
        return out

    def table_size(self):
        return self.L.ohi_table_size(self.p)

    def inflate_block(self, block):
        import ctypes
        b = bytes(block)
        acap = 64 * len(b) + 8 * 4096 + 64
        nvcap = len(b) + 16
        arena = ctypes.create_string_buffer(acap)
        nv = (ctypes.c_uint32 * (5 * nvcap))()
        au, nu = ctypes.c_size_t(), ctypes.c_size_t()
        bb = ctypes.create_string_buffer(b, max(1, len(b)))
        rv = self.L.ohi_inflate_block(self.p, bb, len(b), arena, acap, ctypes.byref(au), nv, nvcap,
                                      ctypes.byref(nu))
        assert rv != -2, "buffers"
        raw = arena.raw[:au.value]
        fields = [(raw[nv[5 * k]:nv[5 * k] + nv[5 * k + 1]],
                   raw[nv[5 * k + 2]:nv[5 * k + 2] + nv[5 * k + 3]], nv[5 * k + 4])
                  for k in range(nu.value)]
        return int(rv), fields


def c_inflate_batch_timed(blocks, conns, nconn, nthreads):
    """Inflate `blocks` (block i on connection conns[i]) with fresh C
    inflaters on `nthreads` threads; returns (seconds, fields)."""
    import ctypes
    L = _clib()
    m = len(blocks)
    keep = [ctypes.create_string_buffer(bytes(b), max(1, len(b))) for b in blocks]
    ptrs = (ctypes.c_void_p * m)(*[ctypes.cast(k, ctypes.c_void_p) for k in keep])
    lens = (ctypes.c_size_t * m)(*[len(b) for b in blocks])
    cs = (ctypes.c_uint32 * m)(*conns)
    nf = ctypes.c_long()
    dt = L.ohi_inflate_batch_timed(ptrs, lens, cs, m, nconn, nthreads, ctypes.byref(nf))
    assert dt >= 0 and nf.value >= 0
    return dt, nf.value
