#!/usr/bin/env python3
"""Per-kernel GPU time of the LAST query of a rocprofv3 kernel trace.

usage: kernel_mix.py <kernel_trace.csv> [window_ms]

The window is the last ``window_ms`` (default: the bench's ms_per_step
is not known here, so 300 ms) of kernel activity.  Kernels are grouped by a
short name (the lambda / kernel identifier without template arguments);
'busy' is the union of kernel intervals (concurrent kernels overlap, so
the per-kernel sums can exceed it).
"""
import csv
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"(dx_[a-z0-9_]+)::\{lambda", name)
    if m:
        return m.group(1)
    m = re.search(r"(?:namespace\)::|^|\s)([A-Za-z_][A-Za-z0-9_]*(?:<\d+>)?)\(", name)
    if m and m.group(1) not in ("void", "operator"):
        return m.group(1)
    return name[:60]


def main():
    path = sys.argv[1]
    win = float(sys.argv[2]) if len(sys.argv) > 2 else 300.0
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         int(r.get("Scratch_Size") or 0), int(r.get("VGPR_Count") or 0)))
    end = max(e for _, e, _, _, _ in rows)
    lo = end - win * 1e6
    sel = [r for r in rows if r[0] >= lo]
    agg = defaultdict(lambda: [0.0, 0, 0, 0])
    for s, e, n, scr, vg in sel:
        a = agg[short(n)]
        a[0] += (e - s) / 1e6
        a[1] += 1
        a[2] = max(a[2], scr)
        a[3] = max(a[3], vg)
    iv = sorted((s, e) for s, e, _, _, _ in sel)
    busy, cur_s, cur_e = 0.0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += (cur_e - cur_s) / 1e6
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += (cur_e - cur_s) / 1e6
    print(f"window {win:.0f} ms, {len(sel)} kernels, GPU busy (union) {busy:.1f} ms")
    print(f"{'ms':>9} {'calls':>6} {'scratch':>8} {'vgpr':>5}  kernel")
    for k, (ms, c, scr, vg) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:45]:
        print(f"{ms:9.2f} {c:6d} {scr:8d} {vg:5d}  {k}")


if __name__ == "__main__":
    main()
