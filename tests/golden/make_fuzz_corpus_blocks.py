#!/usr/bin/env python3
"""Extract the HPACK header blocks of the reference's fuzz corpus into
tests/golden/fuzz_corpus_blocks.json (run in the build container, where
/root/reference exists; the GPU box only reads the JSON).

The corpus (`fuzz/corpus/h2spec`, 133 files, and `fuzz/corpus/nghttp`, 3
files) holds HTTP/2 client connections -- the connection preface, then
frames -- that `fuzz/fuzz_target.cc` feeds to a server session
(`nghttp2_session_mem_recv2`), whose inflater decodes every header block in
arrival order (`lib/nghttp2_session.c` inflate_header_block ->
`nghttp2_hd_inflate_hd3`).  This script does frame parsing only (RFC 9113
section 4.1 frame layout, section 6.2 / 6.6 / 6.10 for HEADERS, PUSH_PROMISE
and CONTINUATION): per file, the header block fragments of each HEADERS or
PUSH_PROMISE frame with its CONTINUATION frames up to END_HEADERS, padding
and priority fields removed, in file order.  No session semantics are
applied (stream states, SETTINGS, connection errors): the test feeds every
block of a file to one inflater, as one connection, and compares the batched
front-end with the oracle block by block, errors and all.  The JSON holds
data only: per file its name, the block bytes (hex), and what the parse
dropped (a block cut by a frame other than CONTINUATION, a frame cut by the
end of the file, a padding length past the payload).
"""
import json
import os
import sys

REF = "/root/reference/fuzz/corpus"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fuzz_corpus_blocks.json")
PREFACE = b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n"
HEADERS, PUSH_PROMISE, CONTINUATION = 0x1, 0x5, 0x9
END_HEADERS, PADDED, PRIORITY = 0x4, 0x8, 0x20


def frames(data):
    """(type, flags, stream, payload) of each whole frame, and whether the
    file ended inside one."""
    p = len(PREFACE) if data.startswith(PREFACE) else 0
    out = []
    while p + 9 <= len(data):
        ln = int.from_bytes(data[p:p + 3], "big")
        ty, fl = data[p + 3], data[p + 4]
        sid = int.from_bytes(data[p + 5:p + 9], "big") & 0x7FFFFFFF
        if p + 9 + ln > len(data):
            return out, True
        out.append((ty, fl, sid, data[p + 9:p + 9 + ln]))
        p += 9 + ln
    return out, p != len(data)


def fragment(ty, fl, payload):
    """The header block fragment of a HEADERS / PUSH_PROMISE frame, or None
    when its padding length passes the payload."""
    q, end = 0, len(payload)
    if fl & PADDED:
        if not payload:
            return None
        pad = payload[0]
        q = 1
        end -= pad
    if ty == HEADERS and fl & PRIORITY:
        q += 5
    if ty == PUSH_PROMISE:
        q += 4
    if q > end:
        return None
    return payload[q:end]


def blocks_of(data):
    fr, cut = frames(data)
    blocks, dropped = [], {"interrupted": 0, "bad_padding": 0, "truncated_frame": int(cut)}
    cur = None
    for ty, fl, sid, pl in fr:
        if cur is not None:
            if ty == CONTINUATION:
                cur += pl
                if fl & END_HEADERS:
                    blocks.append(bytes(cur))
                    cur = None
                continue
            dropped["interrupted"] += 1
            cur = None
        if ty in (HEADERS, PUSH_PROMISE):
            f = fragment(ty, fl, pl)
            if f is None:
                dropped["bad_padding"] += 1
                continue
            if fl & END_HEADERS:
                blocks.append(bytes(f))
            else:
                cur = bytearray(f)
    if cur is not None:
        dropped["interrupted"] += 1
    return blocks, dropped


def main():
    if not os.path.isdir(REF):
        sys.exit("the reference corpus is not here (%s): run in the build container" % REF)
    conns = []
    for sub in ("h2spec", "nghttp"):
        d = os.path.join(REF, sub)
        for name in sorted(os.listdir(d)):
            with open(os.path.join(d, name), "rb") as f:
                data = f.read()
            blocks, dropped = blocks_of(data)
            conns.append({"corpus": sub, "file": name, "bytes": len(data),
                          "blocks": [b.hex() for b in blocks], "dropped": dropped})
    with open(OUT, "w") as f:
        json.dump({"source": "reference fuzz/corpus/{h2spec,nghttp} (fuzz/fuzz_target.cc inputs); "
                             "header blocks by tests/golden/make_fuzz_corpus_blocks.py",
                   "connections": conns}, f, indent=0)
    nb = sum(len(c["blocks"]) for c in conns)
    print("%d connections, %d header blocks, %d bytes of blocks -> %s"
          % (len(conns), nb, sum(len(b) // 2 for c in conns for b in c["blocks"]), OUT))


if __name__ == "__main__":
    main()
