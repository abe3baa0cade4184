#!/usr/bin/env python3
"""Per-kernel GPU time of the LAST query in a rocprofv3 kernel trace (CSV):
queries start at the first ElGamal encryption after a >100 ms gap (as
gpu_busy.py).  With AMD_SERIALIZE_KERNEL=3 the durations are each kernel's
cost alone on the chip (no overlap inflation).  Usage: kernel_cost.py trace.csv [--inner]
--inner: the second-to-last query, bounded by the last query's start (the
last window also holds whatever the program runs after its timed steps)."""
import csv
import sys
from collections import defaultdict


def _name(n: str) -> str:
    n = n.replace("(anonymous namespace)::", "")
    if "for_each_kernel" in n and "<" in n:
        return n.split("<", 1)[1].split("::")[0]
    return n.split("(")[0][:70]


rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
enc = [s for s, e, n in iv if "dx_elgamal_encrypt" in n]
starts = [enc[0]] + [b for a, b in zip(enc, enc[1:]) if b - a > 100e6]
inner = "--inner" in sys.argv and len(starts) > 1
t0, t1 = (starts[-2], starts[-1]) if inner else (starts[-1], float("inf"))
agg = defaultdict(lambda: [0, 0.0])
for s, e, n in iv:
    if t0 <= s < t1:
        a = agg[_name(n)]
        a[0] += 1
        a[1] += (e - s) / 1e6
tot = sum(v[1] for v in agg.values())
nk = sum(v[0] for v in agg.values())
print(f"{'inner' if inner else 'last'} query: {nk} kernels, {tot:.1f} ms of kernel time (serialized)")
print(f"{'ms':>8} {'n':>6}  kernel")
for k, (c, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{ms:8.2f} {c:6d}  {k}")
