#!/usr/bin/env python3
"""Per-kernel duration stats from a rocprofv3 results .db (kernels view):
name, calls, mean/median/min us, in dispatch order of first appearance.
Usage: kstat_db.py <dir or db> [name filter]"""
import glob, os, sqlite3, sys
import numpy as np
p = sys.argv[1]
db = p if p.endswith(".db") else glob.glob(os.path.join(p, "*.db"))[0]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
c = sqlite3.connect(db)
rows = c.execute("select name, duration, grid_x, workgroup_x, vgpr_count, lds_size from kernels order by start").fetchall()
order, d = [], {}
for name, dur, gx, wx, vg, lds in rows:
    key = name.split("(")[0] + ("" if "<" not in name.split("(")[0] else "")
    key = name[:90]
    if flt and flt not in name:
        continue
    if key not in d:
        d[key] = []
        order.append((key, gx, wx, vg, lds))
    d[key].append(dur / 1000.0)
for key, gx, wx, vg, lds in order:
    v = np.array(d[key])
    print("%-90s n=%3d mean=%9.1f med=%9.1f min=%9.1f  grid=%d wg=%d vgpr=%d lds=%d" % (
        key, len(v), v.mean(), np.median(v), v.min(), gx, wx, vg, lds))
