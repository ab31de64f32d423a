#!/usr/bin/env python3
"""Config 1 (BASELINE.json configs[0]): deflatehd -> inflatehd round trip of
the 1,000-case hpack-test-case set (tests/golden/config1_cases.json).

Runs the batched drivers (nghttp2_amd/bin) --timing, REPS times each, and
reports the best time of the batched library calls (the drivers' own JSON
parsing and printing excluded, as they are the reference tools' too), plus
the whole-process wall time.  Also checks the wire against the committed
expected wire.  The CPU line is the Python restatement
(oracle/hpack_oracle.py) doing the same round trip, one core: a
behavioural baseline only, since the reference tools cannot be built here
(C++23 <print>, jansson).  Prints one JSON object."""
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
BIN = os.path.join(REPO, "nghttp2_amd", "bin")
SRC = os.path.join(REPO, "tests", "golden", "config1_cases.json")
REPS = 7


def timed(tool, args, stdin=None):
    t0 = time.perf_counter()
    p = subprocess.run([os.path.join(BIN, tool), *args, "--timing", "--repeat", "10"], input=stdin,
                       capture_output=True, timeout=120, check=True)
    wall = time.perf_counter() - t0
    tline = [ln for ln in p.stderr.decode().splitlines() if ln.startswith('{"timing"')][-1]
    return p.stdout, json.loads(tline)["timing"], wall


def many(nconn=64):
    """The same set as nconn independent connections (files) in one batch."""
    import shutil
    import tempfile
    d = tempfile.mkdtemp(prefix="cfg1_")
    try:
        files = []
        for k in range(nconn):
            f = os.path.join(d, "c%03d.json" % k)
            shutil.copyfile(SRC, f)
            files.append(f)
        os.mkdir(os.path.join(d, "w"))
        os.mkdir(os.path.join(d, "h"))
        _, td, _ = timed("deflatehd", ["-o", os.path.join(d, "w")] + files)
        wf = [os.path.join(d, "w", os.path.basename(f)) for f in files]
        _, ti, _ = timed("inflatehd", ["-o", os.path.join(d, "h")] + wf)
        raw = td["input_bytes"]
        rt = td["warm_seconds"] + ti["warm_seconds"]
        return {"connections": nconn, "cases": td["blocks"], "header_bytes": raw,
                "warm_deflate_call_s": round(td["warm_seconds"], 6),
                "warm_inflate_call_s": round(ti["warm_seconds"], 6),
                "warm_roundtrip_header_MBps": round(raw / rt / 1e6, 2)}
    finally:
        shutil.rmtree(d)


def main():
    gold = json.load(open(os.path.join(REPO, "tests", "golden", "config1_wire.json")))["wire"]
    best = {"deflate": None, "inflate": None}
    walls = {"deflate": [], "inflate": []}
    for _ in range(REPS):
        out, td, wd = timed("deflatehd", [SRC])
        assert [c["wire"] for c in json.loads(out)["cases"]] == gold
        _, ti, wi = timed("inflatehd", [], stdin=out)
        for k, t, w in (("deflate", td, wd), ("inflate", ti, wi)):
            walls[k].append(w)
            if best[k] is None or t["seconds"] < best[k]["seconds"]:
                best[k] = t
    warm = {k: best[k]["warm_seconds"] for k in best}
    raw = best["deflate"]["input_bytes"]
    wire = best["deflate"]["wire_bytes"]
    rt = best["deflate"]["seconds"] + best["inflate"]["seconds"]

    from oracle import hpack_oracle as HO
    cases = json.load(open(SRC))["cases"]
    lists = [[(k.encode(), v.encode()) for p in c["headers"] for k, v in p.items()] for c in cases]
    t0 = time.perf_counter()
    d, inf = HO.Deflater(), HO.Inflater()
    for hl in lists:
        inf.inflate_block(d.deflate_block(hl))
    cpu = time.perf_counter() - t0
    print(json.dumps({
        "config": "1: deflatehd -> inflatehd round trip, 1000-case hpack-test-case set, 1 connection",
        "cases": len(cases), "header_bytes": raw, "wire_bytes": wire,
        "deflate_call_s": round(best["deflate"]["seconds"], 6),
        "inflate_call_s": round(best["inflate"]["seconds"], 6),
        "roundtrip_call_s": round(rt, 6),
        "roundtrip_header_MBps": round(raw / rt / 1e6, 2),
        "roundtrip_cases_per_s": round(len(cases) / rt),
        "warm_deflate_call_s": round(warm["deflate"], 6),
        "warm_inflate_call_s": round(warm["inflate"], 6),
        "warm_roundtrip_header_MBps": round(raw / (warm["deflate"] + warm["inflate"]) / 1e6, 2),
        "many_connections": many(),
        "process_wall_s": {k: round(min(v), 4) for k, v in walls.items()},
        "wire_equals_expected": True,
        "cpu_restatement": {"kind": "port (Python restatement)", "cores": 1,
                            "roundtrip_s": round(cpu, 4),
                            "roundtrip_header_MBps": round(raw / cpu / 1e6, 3)},
    }, indent=1))


if __name__ == "__main__":
    main()
