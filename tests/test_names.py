"""Header-name tokens and FNV-1a name hash.

CPU: the oracle (oracle/hpack_oracle.py lookup_token / name_hash) is pinned to
the reference's own data (tests/golden/name_tokens.json: every name
lookup_token returns a token for, lib/nghttp2_hd.c:137-520, and the static
table's precomputed hashes, :62-126), and the library's host lookup
(nghttp2_amd_hd_lookup_token / _name_hash, no GPU call) matches it.
GPU: nghttp2_amd_hd_name_tokens_batch (k_name_tokens) vs the oracle,
bit-exact, including waves whose names exceed the LDS staging region.
"""
import json
import os

import numpy as np
import pytest

from oracle import hpack_oracle as H
from nghttp2_amd import hd
from nghttp2_amd.workloads import TOKEN_NAMES, gen_names, names_to_pool

GOLD = os.path.join(os.path.dirname(__file__), "golden", "name_tokens.json")


def _gold():
    with open(GOLD) as f:
        return json.load(f)


def _names(pool, off):
    return [pool[off[i]:off[i + 1]].tobytes() for i in range(len(off) - 1)]


def test_oracle_pinned_to_reference_tokens():
    g = _gold()
    assert len(g["tokens"]) == 59
    for name, tok in g["tokens"]:
        assert H.lookup_token(name.encode()) == tok, name
    assert sorted(H._TOKENS.values()) == sorted(t for _, t in g["tokens"])


def test_oracle_pinned_to_reference_static_hashes():
    for name, h in _gold()["static_hashes"]:
        assert H.name_hash(name.encode()) == h, name


def test_workload_token_names_are_the_reference_set():
    assert sorted(n.encode() for n, _ in _gold()["tokens"]) == sorted(TOKEN_NAMES)


def test_host_lookup_matches_golden_and_oracle():
    for name, tok in _gold()["tokens"]:
        assert hd.lookup_token(name.encode()) == tok
        assert hd.name_hash(name.encode()) == H.name_hash(name.encode())
    pool, off = gen_names(4096, seed=7)
    for nm in _names(pool, off):
        assert hd.lookup_token(nm) == H.lookup_token(nm), nm
        assert hd.name_hash(nm) == H.name_hash(nm), nm


def test_host_lookup_edges():
    assert hd.lookup_token(b"") == -1
    assert hd.name_hash(b"") == 2166136261
    assert hd.lookup_token(b"TE") == -1          # case-sensitive, as memeq
    assert hd.lookup_token(b"te") == 61
    assert hd.lookup_token(b":status") == 7      # first static index
    assert hd.lookup_token(b":statu") == -1
    assert hd.lookup_token(b"content-type\x00") == -1


# ---------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------
def _gpu_tokens(codec, dev, pool, off):
    import torch
    n = len(off) - 1
    used = int(off[-1])
    buf = np.zeros(used + (-used) % 16 + 16, dtype=np.uint8)
    buf[:used] = pool[:used]
    names = torch.from_numpy(buf).to(dev)
    noff = torch.from_numpy(np.ascontiguousarray(off).view(np.int32)).to(dev)
    tok, h = codec.name_tokens(names, noff)
    torch.cuda.synchronize()
    return tok.cpu().numpy()[:n], h.cpu().numpy().view(np.uint32)[:n]


def _check(codec, dev, pool, off):
    tok, h = _gpu_tokens(codec, dev, pool, off)
    et, eh = H.name_tokens(_names(pool, off))
    np.testing.assert_array_equal(tok, np.array(et, dtype=np.int32))
    np.testing.assert_array_equal(h, np.array(eh, dtype=np.uint32))


@pytest.mark.gpu
def test_gpu_reference_token_set(codec, dev):
    names = [n.encode() for n, _ in _gold()["tokens"]]
    _check(codec, dev, *names_to_pool(names))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 63, 64, 65, 257, 20000])
def test_gpu_mixed_names(codec, dev, n):
    _check(codec, dev, *gen_names(n, seed=n, long_frac=0.1))


@pytest.mark.gpu
def test_gpu_edges(codec, dev):
    names = ([b""] * 70 + [b"te", b"TE", b"t", b"te\x00", b":status", b":statusx"] +
             [bytes(range(256)) * 3] * 64 +            # a wave beyond the staging region
             [b"x" * 2000, b"", b"cookie"] + [b"a"] * 61)
    _check(codec, dev, *names_to_pool(names))


@pytest.mark.gpu
def test_gpu_full_size(codec, dev):
    _check(codec, dev, *gen_names(1 << 20))
