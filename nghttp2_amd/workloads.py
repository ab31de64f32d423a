"""Synthetic batched header-string workloads (BASELINE.json configs 2-5).

Deterministic numpy generators (PCG64 with the SURVEY.md 8(d) seeds).  A
batch is SoA: a uint8 pool padded to a multiple of 16 bytes and uint32
offsets[n+1].

Also holds a vectorised numpy Huffman bit-packer (`pack_symbols`) used only
to synthesise the decode-only adversarial batch (config 5), whose strings
include EOS codes and malformed padding that no encoder emits.  It is not
the product encoder (that is the HIP library) and not the oracle.
"""
import numpy as np

SEED = {2: 0x5EED0002, 3: 0x5EED0003, 4: 0x5EED0004, 5: 0x5EED0005}

# RFC 7541 Appendix B code lengths (same data as nghttp2_amd/tools/gen_tables.py)
from .tools.gen_tables import RFC7541_LEN, canonical_codes  # noqa: E402

_CODES, _ = canonical_codes()
CODE_VAL = np.array([c for c, _ in _CODES], dtype=np.uint64)
CODE_LEN = np.array(RFC7541_LEN, dtype=np.int64)

PSEUDO_ALPHABET = np.frombuffer(
    b"abcdefghijklmnopqrstuvwxyz0123456789/:._-?=&%ABCDEFGHIJKLMNOPQRSTUVWXYZ",
    dtype=np.uint8)
_PSEUDO_W = np.array([3.0] * 26 + [2.0] * 10 + [2.0] * 9 + [1.0] * 26)
COOKIE_ALPHABET = np.frombuffer(
    b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/=;,-_%",
    dtype=np.uint8)
PRINTABLE = np.arange(0x20, 0x7F, dtype=np.uint8)


def _pool_from_lengths(lengths, chars):
    n = len(lengths)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lengths, out=off[1:])
    total = int(off[-1])
    assert total < 2**32, "pool exceeds uint32 offsets; shard the batch"
    pad = (-total) % 16 + 16
    pool = np.zeros(total + pad, dtype=np.uint8)
    pool[:total] = chars[:total]
    return pool, off.astype(np.uint32)


def gen_pseudo_headers(n, seed=SEED[2], lo=8, hi=64):
    """Config 2: n strings, length uniform in [lo, hi], pseudo-header
    alphabet ([a-z0-9/:._-?=&%] plus upper case)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lengths = rng.integers(lo, hi + 1, size=n, dtype=np.int64)
    p = _PSEUDO_W / _PSEUDO_W.sum()
    chars = rng.choice(PSEUDO_ALPHABET, size=int(lengths.sum()), p=p)
    return _pool_from_lengths(lengths, chars)


def zipf_lengths(rng, n, lo=16, hi=1024, s=1.0):
    ranks = np.arange(1, hi - lo + 2, dtype=np.float64)
    w = ranks ** (-s)
    w /= w.sum()
    return lo + rng.choice(len(ranks), size=n, p=w).astype(np.int64)


def gen_mixed_values(n, seed=SEED[3], lo=16, hi=1024):
    """Config 3/4: n values, Zipf(s=1) over length rank in [lo, hi];
    printable ASCII weighted toward base64/cookie characters."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lengths = zipf_lengths(rng, n, lo, hi)
    total = int(lengths.sum())
    cookie = rng.choice(COOKIE_ALPHABET, size=total)
    other = rng.choice(PRINTABLE, size=total)
    pick = rng.random(total) < 0.85
    chars = np.where(pick, cookie, other).astype(np.uint8)
    return _pool_from_lengths(lengths, chars)


CHUNK = 1 << 16  # strings per independently seeded generation chunk


def mixed_lengths(n, seed=SEED[4], lo=16, hi=1024):
    """Config-4 lengths for all n strings (cheap), chunk-seeded."""
    out = np.empty(n, dtype=np.int64)
    for c0 in range(0, n, CHUNK):
        rng = np.random.Generator(np.random.PCG64([seed, c0 // CHUNK]))
        out[c0:c0 + CHUNK] = zipf_lengths(rng, min(CHUNK, n - c0), lo, hi)
    return out


def _mixed_chunk(lengths, c, s0, s1, seed):
    c0, c1 = c * CHUNK, min((c + 1) * CHUNK, len(lengths))
    rng = np.random.Generator(np.random.PCG64([seed, 1 << 20, c]))
    tot = int(lengths[c0:c1].sum())
    cookie = rng.choice(COOKIE_ALPHABET, size=tot)
    other = rng.choice(PRINTABLE, size=tot)
    chars = np.where(rng.random(tot) < 0.85, cookie, other).astype(np.uint8)
    cum = np.concatenate([[0], np.cumsum(lengths[c0:c1])])
    a, b = max(s0, c0) - c0, min(s1, c1) - c0
    return chars[cum[a]:cum[b]]


def gen_mixed_range(lengths, s0, s1, seed=SEED[4], threads=1):
    """Characters of strings [s0, s1) of a chunk-seeded config-4 set: each
    rank generates only its own shard.  Returns (pool, off) rebased to 0.
    The chunks are seeded independently, so `threads` > 1 (a thread pool;
    numpy releases the GIL in the generators) gives the same bytes."""
    chunks = list(range(s0 // CHUNK, (max(s1, s0 + 1) - 1) // CHUNK + 1))
    if threads > 1 and len(chunks) > 1:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(threads) as ex:
            parts = list(ex.map(lambda c: _mixed_chunk(lengths, c, s0, s1, seed), chunks))
    else:
        parts = [_mixed_chunk(lengths, c, s0, s1, seed) for c in chunks]
    chars = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    return _pool_from_lengths(lengths[s0:s1], chars)


def gen_all_bytes(n, seed=1, lo=0, hi=64):
    """Uniformly random bytes 0..255 (exercises every code length)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lengths = rng.integers(lo, hi + 1, size=n, dtype=np.int64)
    chars = rng.integers(0, 256, size=int(lengths.sum()), dtype=np.uint8)
    return _pool_from_lengths(lengths, chars)


def pack_symbols(sym_pool, sym_off, pad_bits_value=None):
    """Vectorised MSB-first packing of symbol strings (0..256, 256 = EOS).

    Returns (enc_pool, enc_off, pad) where each string is padded to a byte
    boundary; pad_bits_value(i, npad) is not supported -- padding is all
    ones (the EOS prefix, as lib/nghttp2_hd_huffman.c:95-101) and callers
    corrupt it afterwards for adversarial cases.  pad[i] = number of pad bits.
    """
    sym_pool = np.asarray(sym_pool, dtype=np.int64)
    sym_off = np.asarray(sym_off, dtype=np.int64)
    n = len(sym_off) - 1
    L = CODE_LEN[sym_pool]
    bits_per_str = np.add.reduceat(np.append(L, 0), sym_off[:-1]) if len(L) else np.zeros(n, np.int64)
    empty = sym_off[1:] == sym_off[:-1]
    bits_per_str = np.where(empty, 0, bits_per_str).astype(np.int64)
    enc_len = (bits_per_str + 7) // 8
    pad = enc_len * 8 - bits_per_str
    enc_off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(enc_len, out=enc_off[1:])
    total = int(enc_off[-1])
    # global bit position of every symbol
    cum = np.cumsum(L) - L  # exclusive over the whole pool
    str_of_sym = np.repeat(np.arange(n), np.diff(sym_off))
    start_of_str_bits = (cum[sym_off[:-1][~empty]] if len(L) else np.zeros(0, np.int64))
    base = np.zeros(n, dtype=np.int64)
    base[~empty] = start_of_str_bits
    P = enc_off[str_of_sym] * 8 + (cum - base[str_of_sym])
    byte0 = P >> 3
    sh = P & 7
    v = CODE_VAL[sym_pool].astype(np.uint64) << (np.uint64(40) - L.astype(np.uint64)
                                                 - sh.astype(np.uint64))
    out = np.zeros(total + 8, dtype=np.float64)
    for k in range(5):
        part = ((v >> np.uint64(32 - 8 * k)) & np.uint64(0xFF)).astype(np.float64)
        out += np.bincount(byte0 + k, weights=part, minlength=total + 8)
    enc = out.astype(np.uint8)
    has_pad = pad > 0
    last = enc_off[1:] - 1
    enc[last[has_pad]] |= ((1 << pad[has_pad]) - 1).astype(np.uint8)
    pool = np.zeros(total + (-total) % 16 + 16, dtype=np.uint8)
    pool[:total] = enc[:total]
    return pool, enc_off.astype(np.uint32), pad


def gen_adversarial(n, seed=SEED[5], return_nsym=False):
    """Config 5: decode-only adversarial batch.  Category per string (id in
    cats[i]): 0 valid 30-bit symbols (10, 13, 22) + 28-bit control bytes;
    1 embedded EOS; 2 padding of 8-15 ones; 3 zero-bit padding; 4 truncated
    long code; 5 valid text with 0-7 bit all-ones padding; 6 empty;
    7 random bytes.  Returns (enc_pool, enc_off, cats[, nsym]); nsym[i] is
    the number of symbols packed into string i before any corruption (the
    decoded length of a valid string).  Vectorised; the random draws keep
    the order of the original per-string generator, so a seed gives the
    same batch."""
    rng = np.random.Generator(np.random.PCG64(seed))
    cats = rng.integers(0, 8, size=n)
    nsym = rng.integers(1, 24, size=n)
    nsym[cats == 6] = 0
    sym_off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(nsym, out=sym_off[1:])
    tot = int(sym_off[-1])
    str_of = np.repeat(np.arange(n), nsym)
    c_of = cats[str_of]
    long_syms = np.array([10, 13, 22, 0, 1, 2, 3, 4, 5, 6, 7, 8, 11, 12, 14, 127, 220, 249],
                         dtype=np.int64)
    text = rng.choice(np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789-_./", np.uint8),
                      size=tot).astype(np.int64)
    syms = np.where(np.isin(c_of, [0, 4]), rng.choice(long_syms, size=tot), text)
    # category 1: one symbol replaced by EOS
    first = sym_off[:-1]
    eos_pos = first + (rng.integers(0, 1 << 30, size=n) % np.maximum(nsym, 1))
    m = (cats == 1) & (nsym > 0)
    syms[eos_pos[m]] = 256
    pool, enc_off, pad = pack_symbols(syms, sym_off)
    enc_off = enc_off.astype(np.int64)
    L = np.diff(enc_off)
    new_len = L.copy()
    c2 = (cats == 2) & (L > 0)  # one more 0xFF byte: the pad becomes 8..15 ones
    c3 = (cats == 3) & (L > 0) & (pad > 0)  # zero-bit padding
    c4 = (cats == 4) & (L > 1)  # cut inside the trailing 28/30-bit code
    r7 = np.nonzero(cats == 7)[0]  # random bytes
    new_len[c2] += 1
    new_len[c4] -= 1
    rand7 = []
    for _ in r7:
        k = int(rng.integers(1, 40))
        rand7.append(rng.integers(0, 256, size=k, dtype=np.uint8))
    new_len[r7] = [len(x) for x in rand7]
    out_off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(new_len, out=out_off[1:])
    allb = np.zeros(int(out_off[-1]), dtype=np.uint8)

    def spans(starts, lens):  # concatenated index ranges [starts[i], starts[i] + lens[i])
        tot = int(lens.sum())
        return np.repeat(starts, lens) + (np.arange(tot) - np.repeat(np.cumsum(lens) - lens, lens))

    cl = np.where(cats != 7, np.minimum(L, new_len), 0)
    allb[spans(out_off[:-1], cl)] = pool[spans(enc_off[:-1], cl)]
    allb[out_off[1:][c2] - 1] = 0xFF
    allb[out_off[1:][c3] - 1] &= ((0xFF << pad[c3]) & 0xFF).astype(np.uint8)
    if len(r7):
        allb[spans(out_off[r7], new_len[r7])] = np.concatenate(rand7)
    out_pool, out_off = _pool_from_lengths(new_len, allb)
    if return_nsym:
        return out_pool, out_off, cats, nsym
    return out_pool, out_off, cats


# Header names for the token / name-hash batch.
TOKEN_NAMES = [
    b":authority", b":method", b":path", b":scheme", b":status", b"accept-charset",
    b"accept-encoding", b"accept-language", b"accept-ranges", b"accept",
    b"access-control-allow-origin", b"age", b"allow", b"authorization", b"cache-control",
    b"content-disposition", b"content-encoding", b"content-language", b"content-length",
    b"content-location", b"content-range", b"content-type", b"cookie", b"date", b"etag",
    b"expect", b"expires", b"from", b"host", b"if-match", b"if-modified-since",
    b"if-none-match", b"if-range", b"if-unmodified-since", b"last-modified", b"link",
    b"location", b"max-forwards", b"proxy-authenticate", b"proxy-authorization", b"range",
    b"referer", b"refresh", b"retry-after", b"server", b"set-cookie",
    b"strict-transport-security", b"transfer-encoding", b"user-agent", b"vary", b"via",
    b"www-authenticate", b"te", b"connection", b"keep-alive", b"proxy-connection", b"upgrade",
    b":protocol", b"priority"]
_NAME_ALPHABET = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789-_", dtype=np.uint8)


def gen_names(n, seed=0x5EED0006, long_frac=0.02):
    """n header names: ~55% token names, ~12% near misses (one byte changed,
    upper-cased, cut or extended by a byte), ~30% random x-/custom names of
    1..40 bytes, ~3% empty; and whole waves (64 aligned names) of long names
    (100..600 B) with probability long_frac, which exceed the kernel's
    staging region.  Returns (pool, off)."""
    rng = np.random.default_rng(seed)
    kind = rng.choice(4, size=n, p=[0.55, 0.12, 0.30, 0.03])
    nw = (n + 63) // 64
    long_wave = rng.random(nw) < long_frac
    kind[np.repeat(long_wave, 64)[:n]] = 4
    pick = rng.integers(0, len(TOKEN_NAMES), size=n)
    lens = np.where(kind == 4, rng.integers(100, 601, size=n), rng.integers(1, 41, size=n))
    rnd = _NAME_ALPHABET[rng.integers(0, len(_NAME_ALPHABET), size=int(lens.sum()))].tobytes()
    roff = np.concatenate([[0], np.cumsum(lens)])
    mut = rng.integers(0, 4, size=n)
    pos = rng.integers(0, 1 << 30, size=n)
    bit = rng.integers(0, 7, size=n)
    out = []
    for i in range(n):
        k = kind[i]
        if k == 0:
            out.append(TOKEN_NAMES[pick[i]])
        elif k == 1:
            b = bytearray(TOKEN_NAMES[pick[i]])
            m = mut[i]
            if m == 0:
                b[pos[i] % len(b)] ^= 1 << int(bit[i])
            elif m == 1:
                b = bytearray(bytes(b).upper())
            elif m == 2:
                b = b[:-1]
            else:
                b.append(rnd[roff[i]])
            out.append(bytes(b))
        elif k == 2:
            out.append(b"x-" + rnd[roff[i]:roff[i + 1]])
        elif k == 3:
            out.append(b"")
        else:
            out.append(rnd[roff[i]:roff[i + 1]])
    return names_to_pool(out)


def names_to_pool(names):
    lengths = np.array([len(x) for x in names], dtype=np.int64)
    return _pool_from_lengths(lengths, np.frombuffer(b"".join(names), dtype=np.uint8))
