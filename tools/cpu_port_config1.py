#!/usr/bin/env python3
"""The oracle's C inflater (oracle/hpack_inflate_oracle.c) on config 1's
committed wire (tests/golden/config1_wire.json: 1,000 blocks of one
connection), one thread, best of 20: the CPU baseline for the inflatehd
driver's config-1 row."""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import hpack_oracle as HO

d = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden",
                                "config1_wire.json")))
blocks = [bytes.fromhex(x) for x in d["wire"]]
wire = sum(len(b) for b in blocks)
best, nf = None, 0
for _ in range(20):
    dt, nf = HO.c_inflate_batch_timed(blocks, [0] * len(blocks), 1, 1)
    best = dt if best is None or dt < best else best
print(json.dumps({"blocks": len(blocks), "wire_bytes": wire, "fields": nf,
                  "cpu_port_1t_ms": round(best * 1e3, 3), "cpu_port_1t_wire_MBps": round(wire / best / 1e6, 1),
                  "cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": ")}))
