#!/usr/bin/env python3
"""Generate tests/golden/name_tokens.json from the reference's own data.

BUILD-CONTAINER ONLY (reads /root/reference as text; never runs on the GPU
box).  Two vectors, both read out of lib/ as data:

- tokens: every (name, token) lookup_token can return
  (lib/nghttp2_hd.c:137-520: the name is the memeq prefix plus the byte the
  inner switch cases on; the token value comes from the enum in
  lib/nghttp2_hd.h:56-116, explicit for 0..60, consecutive after);
- static_hashes: (name, hash) of the static table's MAKE_STATIC_ENT rows
  (lib/nghttp2_hd.c:62-126), the reference's precomputed FNV-1a values.

Usage: python3 tests/golden/make_name_tokens.py
"""
import json
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/lib"


def token_values():
    text = open(os.path.join(REF, "nghttp2_hd.h")).read()
    body = text[text.index("typedef enum {", text.index("NGHTTP2_TOKEN__AUTHORITY") - 200):]
    body = body[:body.index("}")]
    vals, nxt = {}, 0
    for m in re.finditer(r"(NGHTTP2_TOKEN_\w+)\s*(?:=\s*(\d+))?\s*,", body):
        v = int(m.group(2)) if m.group(2) is not None else nxt
        vals[m.group(1)] = v
        nxt = v + 1
    return vals


def lookup_token_names(vals):
    text = open(os.path.join(REF, "nghttp2_hd.c")).read()
    start = text.index("static int32_t lookup_token(")
    body = text[start:text.index("\n}\n", start)]
    out, last = [], None
    tok = re.compile(r"case '(.)':|memeq\(\"([^\"]*)\", name, (\d+)\)|return (NGHTTP2_TOKEN_\w+)")
    prefix = None
    for m in tok.finditer(body):
        if m.group(1) is not None:
            last = m.group(1)
        elif m.group(2) is not None:
            assert len(m.group(2)) == int(m.group(3))
            prefix = m.group(2)
        else:
            out.append([prefix + last, vals[m.group(4)]])
    return out


def static_hashes():
    text = open(os.path.join(REF, "nghttp2_hd.c")).read()
    return [[n, int(h)] for n, h in re.findall(r'MAKE_STATIC_ENT\("([^"]*)", "[^"]*", \d+, (\d+)u\)', text)]


def main():
    vals = token_values()
    data = {"source": "lib/nghttp2_hd.c:62-126 (static hashes), :137-520 (lookup_token), "
                      "lib/nghttp2_hd.h:56-116 (token values)",
            "tokens": lookup_token_names(vals),
            "static_hashes": static_hashes()}
    assert len(data["static_hashes"]) == 61, len(data["static_hashes"])
    path = os.path.join(HERE, "name_tokens.json")
    with open(path, "w") as f:
        json.dump(data, f, indent=0)
        f.write("\n")
    print("wrote %s: %d tokens, %d static hashes" % (path, len(data["tokens"]), len(data["static_hashes"])))


if __name__ == "__main__":
    main()
