#!/usr/bin/env python3
"""From a rocprofv3 kernel trace of the two-stream bench: the timed steps'
kernels in time order, how long each kernel ran alone or beside another,
and the period per step.  Usage: trace_overlap.py <rocprof dir>"""
import csv, glob, sys
d = sys.argv[1]
rows = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
short = lambda k: ("dec" if "k_decode_items" in k else "enc" if "k_encode" in k else
                   "cnt" if "k_enc_count" in k else k.split("(")[0][-24:])
main = [r for r in rows if short(r[2]) in ("dec", "enc", "cnt")]
# the last 2/3 of the launches (the timed steps come last)
tail = main[len(main) // 3:]
t0, t1 = tail[0][0], tail[-1][1]
ndec = sum(1 for r in tail if short(r[2]) == "dec")
print("launches %d, decodes %d, span %.1f us, per decode-step %.1f us" %
      (len(tail), ndec, (t1 - t0) / 1e3, (t1 - t0) / 1e3 / max(1, ndec)))
# time covered by each set of concurrently running kernel kinds
ev = []
for s, e, k in tail:
    ev.append((s, 1, short(k)))
    ev.append((e, -1, short(k)))
ev.sort()
act = {}
cover = {}
last = ev[0][0]
for t, dlt, k in ev:
    key = "+".join(sorted(x for x, c in act.items() if c > 0)) or "idle"
    cover[key] = cover.get(key, 0) + (t - last)
    last = t
    act[k] = act.get(k, 0) + dlt
tot = sum(cover.values())
for k, v in sorted(cover.items(), key=lambda x: -x[1]):
    print("  %-16s %8.1f us/step  %5.1f %%" % (k, v / 1e3 / max(1, ndec), 100.0 * v / tot))
for kind in ("dec", "enc", "cnt"):
    ds = [(e - s) / 1e3 for s, e, k in tail if short(k) == kind]
    if ds:
        ds.sort()
        print("  %s: median %.1f us (min %.1f, max %.1f) over %d" % (kind, ds[len(ds) // 2], ds[0], ds[-1], len(ds)))
