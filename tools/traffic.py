#!/usr/bin/env python3
"""HBM traffic per launch from the FETCH_SIZE / WRITE_SIZE PMC passes of
tools/gpu_round.sh (gpurun_out/pmc_c<cfg>/p1 = FETCH_SIZE, p2 = WRITE_SIZE).

MI355X_MICROARCH.md (HBM): FETCH_SIZE reports half the bytes of wide
streaming reads on gfx950 (doubled here); WRITE_SIZE reads exact.  Both are
in KiB.  Writes profiles/traffic.json (merged), read by bench.py."""
import csv, glob, json, os, sys
from collections import defaultdict

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
KERNELS = ("k_decode_items", "k_encode", "k_enc_count")


def per_launch(d, counter):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            per[r["Dispatch_Id"]] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for did, v in per.items():
            for k in KERNELS:
                if names[did].startswith(k + "(") or names[did].startswith("void " + k + "<"):
                    acc[k].append(v)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    sys.path.insert(0, ROOT)
    from bench import kernel_src_sha
    src_sha = kernel_src_sha()  # the tree the counters were measured on (bench.py checks it)
    out_path = os.path.join(ROOT, "profiles", "traffic.json")
    res = json.load(open(out_path)) if os.path.exists(out_path) else {}
    for cfg, strings in ((2, 1 << 20), (3, 1 << 20), (5, 1 << 20)):
        base = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out")
        d = os.path.join(base, "pmc_c%d" % cfg)
        if not os.path.isdir(d):
            continue
        fetch = per_launch(os.path.join(d, "p1"), "FETCH_SIZE")
        write = per_launch(os.path.join(d, "p2"), "WRITE_SIZE")
        ent = {}
        for k in KERNELS:
            if k in fetch and k in write:
                rd, wr = 2.0 * fetch[k] * 1024, write[k] * 1024
                ent[k] = {"strings": strings, "read_bytes": int(rd), "write_bytes": int(wr),
                          "src_sha": src_sha,
                          "hbm_bytes_per_launch": int(rd + wr),
                          "source": "%s (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, "
                                    "FETCH x2 per MI355X_MICROARCH.md)" % os.path.relpath(d, ROOT)}
        res.setdefault("config%d" % cfg, {}).update(ent)
    json.dump(res, open(out_path, "w"), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
