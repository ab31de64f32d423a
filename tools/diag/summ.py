#!/usr/bin/env python3
"""Summarise diag outputs (stamps / time_variants JSON, possibly concatenated)."""
import json, sys
txt = "".join(open(p).read() for p in sys.argv[1:])
dec = json.JSONDecoder(); i = 0
while i < len(txt):
    j = txt.find('{', i)
    if j < 0: break
    try:
        o, k = dec.raw_decode(txt[j:])
    except ValueError:
        i = j + 1; continue
    i = j + k
    if 'share' in o:
        print(o['config'], {a: round(b, 3) for a, b in o['share'].items()}, 'iters', round(o['verify_iters_per_round'], 2),
              'mism', round(o['mismatches_per_round'], 2), 'rounds', o['rounds'], 'pass1 cyc/wg', o['cycles_per_wg_median']['pass1'], 'trips', o.get('wave_trips_per_round'), 'wave p1 cyc', o.get('wave_pass1_cycles_per_round'))
    else:
        print(o)
