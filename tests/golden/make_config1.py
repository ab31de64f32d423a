#!/usr/bin/env python3
"""Config 1 (BASELINE.json configs[0]): a 1,000-case hpack-test-case JSON
header set, and the wire nghttp2's deflater produces for it.

The reference ships no such set, so this script
synthesises one: one compression context whose cases alternate browser-like
requests (pseudo-headers, user-agent, accept*, cookie, referer) and responses
(:status, content-type/length, cache-control, date, etag, set-cookie, vary,
server), across a few hosts, with repeated and fresh values so the dynamic
table hits, misses and evicts.  Values are ASCII as JSON headers are.

Outputs (committed):
  tests/golden/config1_cases.json   the input, deflatehd's format
  tests/golden/config1_wire.json    per case the expected wire hex, from the
                                    restated deflater (oracle/hpack_oracle.py,
                                    pinned by RFC 7541 C.4 = nghttp2's output),
                                    and the dynamic table after the last case

Run from the repo root: python3 tests/golden/make_config1.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import hpack_oracle as HO  # noqa: E402

N_CASES = 1000
SEED = 0x5EED0001

ALNUM = np.frombuffer(b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789", np.uint8)


def token(rng, n):
    return bytes(ALNUM[rng.integers(0, len(ALNUM), n)]).decode()


def make_cases():
    rng = np.random.Generator(np.random.PCG64(SEED))
    hosts = ["www.example.com", "static.example.net", "api.example.org", "img.cdn-example.com"]
    uas = ["Mozilla/5.0 (X11; Linux x86_64; rv:128.0) Gecko/20100101 Firefox/128.0",
           "Mozilla/5.0 (Windows NT 10.0; Win64; x64) AppleWebKit/537.36 (KHTML, like Gecko) "
           "Chrome/126.0.0.0 Safari/537.36",
           "curl/8.5.0", "nghttp2/1.70.90"]
    exts = [".html", ".css", ".js", ".png", ".jpg", ".json", ""]
    ctypes = ["text/html; charset=utf-8", "text/css", "application/javascript", "image/png",
              "image/jpeg", "application/json"]
    cookies = ["sid=" + token(rng, 26) for _ in range(6)]
    cases = []
    for i in range(N_CASES):
        host = hosts[int(rng.zipf(1.6)) % len(hosts)]
        if i % 2 == 0:  # request
            path = "/" + "/".join(token(rng, int(rng.integers(3, 12)))
                                  for _ in range(int(rng.integers(1, 4))))
            path += exts[int(rng.integers(0, len(exts)))]
            if rng.random() < 0.3:
                path += "?q=" + token(rng, int(rng.integers(4, 40)))
            h = [{":method": "GET" if rng.random() < 0.85 else "POST"},
                 {":scheme": "https"}, {":authority": host}, {":path": path},
                 {"user-agent": uas[int(rng.integers(0, 2 if rng.random() < 0.9 else 4))]},
                 {"accept": "*/*" if rng.random() < 0.5 else
                  "text/html,application/xhtml+xml,application/xml;q=0.9,*/*;q=0.8"},
                 {"accept-encoding": "gzip, deflate, br"},
                 {"accept-language": "en-US,en;q=0.5"}]
            if rng.random() < 0.7:
                c = cookies[int(rng.integers(0, len(cookies)))]
                if rng.random() < 0.4:
                    c += "; pref=" + token(rng, int(rng.integers(2, 10)))  # short ones never indexed
                h.append({"cookie": c})
            if rng.random() < 0.6:
                h.append({"referer": "https://" + host + "/" + token(rng, int(rng.integers(3, 16)))})
            if rng.random() < 0.15:
                h.append({"x-request-id": token(rng, 32)})
            if rng.random() < 0.05:
                h.append({"authorization": "Bearer " + token(rng, 40)})
        else:  # response
            st = ["200", "200", "200", "304", "404", "301", "500", "204"][int(rng.integers(0, 8))]
            h = [{":status": st},
                 {"date": "Mon, %02d Oct 2026 %02d:%02d:%02d GMT" % (
                     1 + i // 200, (i // 60) % 24, i % 60, int(rng.integers(0, 60)))},
                 {"server": "nghttpx" if rng.random() < 0.8 else "apache"},
                 {"content-type": ctypes[int(rng.integers(0, len(ctypes)))]},
                 {"content-length": str(int(rng.integers(0, 1 << 20)))},
                 {"cache-control": ["private, max-age=0", "public, max-age=31536000",
                                    "no-cache"][int(rng.integers(0, 3))]}]
            if rng.random() < 0.5:
                h.append({"etag": '"' + token(rng, 16) + '"'})
            if rng.random() < 0.2:
                h.append({"set-cookie": "sid=" + token(rng, 26) + "; Path=/; HttpOnly; Secure"})
            if rng.random() < 0.4:
                h.append({"vary": "Accept-Encoding"})
            if rng.random() < 0.1:
                h.append({"x-" + token(rng, int(rng.integers(3, 10))).lower(): token(rng, int(rng.integers(0, 120)))})
        cases.append({"headers": h})
    return {"context": "request", "description": "synthetic config-1 set (tests/golden/make_config1.py)",
            "cases": cases}


def expected(doc, table_size=4096, deflate_table_size=4096):
    d = HO.Deflater(deflate_table_size)
    if table_size != 4096:
        d.change_table_size(table_size)
    wires = []
    for c in doc["cases"]:
        hl = [(k.encode(), v.encode()) for pair in c["headers"] for k, v in pair.items()]
        wires.append(d.deflate_block(hl).hex())
    return wires, [[n.decode(), v.decode()] for n, v in d.table]


def main():
    doc = make_cases()
    wires, table = expected(doc)
    with open(os.path.join(HERE, "config1_cases.json"), "w") as f:
        json.dump(doc, f, indent=0, separators=(",", ":"))
    with open(os.path.join(HERE, "config1_wire.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_config1.py", "deflater": "oracle/hpack_oracle.py",
                   "table_size": 4096, "wire": wires, "final_table": table}, f, indent=0)
    raw = sum(len(k) + len(v) for c in doc["cases"] for p in c["headers"] for k, v in p.items())
    print("cases", len(wires), "header bytes", raw, "wire bytes", sum(len(w) // 2 for w in wires))


if __name__ == "__main__":
    main()
