#!/usr/bin/env python3
"""GPU occupancy per bench step from a rocprofv3 kernel trace: steps start at
the first ElGamal encryption of a query; for each step print wall time, the
union of kernel intervals (GPU busy), idle gaps > 2 ms and the top kernels."""
import csv
import sys
from collections import defaultdict

def _name(n: str) -> str:
    if n.startswith("(anonymous namespace)::"):
        n = n[len("(anonymous namespace)::"):]
    if "for_each_kernel" in n and "<" in n:
        return n.split("<", 1)[1].split("::")[0]
    return n.split("(")[0][:60]


rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
enc = [s for s, e, n in iv if "dx_elgamal_encrypt" in n]
starts = [enc[0]] + [b for a, b in zip(enc, enc[1:]) if b - a > 100e6]
starts.append(iv[-1][1])
for k in range(len(starts) - 1):
    a, b = starts[k], starts[k + 1]
    sel = [(max(s, a), min(e, b), n) for s, e, n in iv if e > a and s < b]
    busy, cur_s, cur_e, gaps = 0, None, None, []
    for s, e, n in sel:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                if s - cur_e > 2e6:
                    gaps.append(((cur_e - a) / 1e6, (s - cur_e) / 1e6))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    tot = defaultdict(float)
    for s, e, n in sel:
        tot[_name(n)] += (e - s) / 1e6
    print(f"step {k}: wall {(b - a) / 1e6:.1f} ms, GPU busy {busy / 1e6:.1f} ms, idle gaps>2ms: "
          + ", ".join(f"@{t:.0f}+{g:.0f}" for t, g in gaps[:12]))
    for nm, t in sorted(tot.items(), key=lambda x: -x[1])[:14]:
        print(f"    {t:8.2f} ms  {nm}")

# timeline of the last full step: long kernels and the gaps before them
if len(sys.argv) > 2:
    a, b = starts[-3], starts[-2]
    prev = a
    print("--- timeline of the last full step (kernels > 1 ms, gaps > 1 ms)")
    for s, e, n in iv:
        if s < a or s > b:
            continue
        if (e - s) > 1e6 or (s - prev) > 1e6:
            print(f"t={(s - a) / 1e6:8.1f} dur={(e - s) / 1e6:7.2f} gap={(s - prev) / 1e6:6.1f} {_name(n)}")
        prev = max(prev, e)
