#!/usr/bin/env python3
"""Pin the oracle (and the product's generated tables) to the reference.

BUILD-CONTAINER ONLY (needs /root/reference; never runs on the GPU box).

1. Runs the reference's own table generator, /root/reference/mkhufftbl.py
   (a Python reference run here, as the oracle rules allow), parses the
   tables it prints, and packs them in the reference struct layouts
   (lib/nghttp2_hd_huffman.h:39-52 and :62-67).
2. Parses the reference's checked-in data file
   lib/nghttp2_hd_huffman_data.c the same way (as data).
3. Checks both byte-for-byte against the oracle's tables
   (oracle/huff_oracle.c) and the product's generator
   (nghttp2_amd/tools/gen_tables.py).
4. Writes tests/golden/reference_tables.json: the sha256 of the reference
   tables, so the CPU test suite can re-check the oracle and the product
   tables without /root/reference present.

Usage: python3 oracle/pin_reference.py
"""
import hashlib
import json
import os
import re
import struct
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
sys.path.insert(0, REPO)


def parse_tables(text):
    sym = re.findall(r"\{\s*(\d+),\s*0x([0-9A-Fa-f]+)U?\s*\}", text)
    dec = re.findall(r"\{\s*0x([0-9A-Fa-f]+),\s*0x([0-9A-Fa-f]+),\s*0x([0-9A-Fa-f]+)\s*\}",
                     text)
    assert len(sym) == 257, len(sym)
    assert len(dec) == 257 * 16, len(dec)
    symb = b"".join(struct.pack("<II", int(n), int(c, 16)) for n, c in sym)
    decb = b"".join(struct.pack("<HBB", int(a, 16), int(b, 16), int(c, 16))
                    for a, b, c in dec)
    return symb, decb


def main():
    gen = subprocess.run([sys.executable, os.path.join(REF, "mkhufftbl.py")],
                         check=True, capture_output=True, text=True, cwd="/tmp").stdout
    ref_sym, ref_dec = parse_tables(gen)
    with open(os.path.join(REF, "lib", "nghttp2_hd_huffman_data.c")) as f:
        data_sym, data_dec = parse_tables(f.read())
    assert (ref_sym, ref_dec) == (data_sym, data_dec), \
        "mkhufftbl.py output differs from lib/nghttp2_hd_huffman_data.c"

    from oracle import oracle
    orc_sym, orc_dec = oracle.tables_ref_layout()
    assert orc_sym == ref_sym, "oracle sym table != reference"
    assert orc_dec == ref_dec, "oracle decode table != reference"

    sys.path.insert(0, os.path.join(REPO, "nghttp2_amd", "tools"))
    import gen_tables
    p_sym, p_dec = gen_tables.packed_ref_layout(gen_tables.build())
    assert p_sym == ref_sym, "product sym table != reference"
    assert p_dec == ref_dec, "product decode table != reference"

    out = {
        "source": "python3 /root/reference/mkhufftbl.py (run in the build container) "
                  "and lib/nghttp2_hd_huffman_data.c parsed as data; identical",
        "layout": "sym: 257 x {u32 nbits, u32 code} LE; dec: 257x16 x {u16 fstate, "
                  "u8 flags, u8 sym} LE (lib/nghttp2_hd_huffman.h:39-67)",
        "sym_sha256": hashlib.sha256(ref_sym).hexdigest(),
        "dec_sha256": hashlib.sha256(ref_dec).hexdigest(),
        "dec_entries": 257 * 16,
    }
    path = os.path.join(REPO, "tests", "golden", "reference_tables.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print("pinned: oracle and product tables == reference;", path)


if __name__ == "__main__":
    main()
