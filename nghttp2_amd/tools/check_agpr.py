#!/usr/bin/env python3
"""Build-time audit of the lane decoder's AGPR chunk staging.

k_decode_lanes stages input chunks in a0..a15 with inline-asm buffer loads
the compiler does not see (csrc/hd_huff.hip, dl_stage_load / dl_stage_read).
That is only safe while no compiler-generated instruction touches a0..a15
between a staged load and the drain after the fast periods
(cdna_hip_programming.md 5.7 item 4: audit after every edit).  This script
reads the device assembly (hipcc --cuda-device-only -S) and fails if, inside
any k_decode_lanes instance, a line outside ;;#ASMSTART/;;#ASMEND names one
of a0..a15 while a staged load may be in flight, or if the kernel spills.

Usage: check_agpr.py <device .s file>
"""
import re
import sys

STAGE = re.compile(r"\ba(?:[0-9]|1[0-5])\b|a\[(\d+):(\d+)\]")


def names_staging(line):
    for m in STAGE.finditer(line):
        if m.group(1) is None:
            return True
        lo, hi = int(m.group(1)), int(m.group(2))
        if lo <= 15:
            return True
    return False


def main(path):
    s = open(path).read()
    bad = []
    kernels = re.findall(r"^(_Z\d+k_decode_lanes\w*):", s, re.M)
    if not kernels:
        print("check_agpr: no k_decode_lanes instance found", file=sys.stderr)
        return 1
    for fn in kernels:
        start = s.index(fn + ":")
        end = s.index(".Lfunc_end", start)
        body = s[start:end].split("\n")
        inasm, inflight = False, False
        for i, line in enumerate(body):
            if ";;#ASMSTART" in line:
                inasm = True
                continue
            if ";;#ASMEND" in line:
                inasm = False
                continue
            if inasm:
                if "buffer_load_dwordx4 a[" in line:
                    inflight = True
                elif "s_waitcnt vmcnt(0)" in line:
                    inflight = False
                continue
            if inflight and names_staging(line.split(";")[0]):
                bad.append("%s+%d: %s" % (fn, i, line.strip()))
        meta = s[s.index(".name:           " + fn):][:4000]
        for key in ("vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size"):
            m = re.search(r"\.%s:\s+(\d+)" % key, meta)
            if m and int(m.group(1)) != 0:
                bad.append("%s: .%s = %s" % (fn, key, m.group(1)))
    if bad:
        print("check_agpr: compiler code touches the staging AGPRs or spills:", file=sys.stderr)
        for b in bad[:20]:
            print("  " + b, file=sys.stderr)
        return 1
    print("check_agpr: %d k_decode_lanes instance(s) clean" % len(kernels))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
