#!/usr/bin/env python3
"""Per-kernel PMC summary of a rocprofv3 --pmc CSV (counter_collection.csv):
dispatches, waves, VALU instructions per wave, the share of the waves'
lifetime spent issuing VALU (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES), LDS
instructions per wave, scratch bytes per lane and VGPRs.  Usage:
pmc_summary.py counter_collection.csv [filter-substring ...]"""
import csv
import sys
from collections import defaultdict


def _name(n: str) -> str:
    if n.startswith("(anonymous namespace)::"):
        n = n[len("(anonymous namespace)::"):]
    if "for_each_kernel" in n and "<" in n:
        return n.split("<", 1)[1].split("::")[0]
    return n.split("(")[0][:60]


agg = defaultdict(lambda: defaultdict(float))
meta = {}
disp = defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = _name(r["Kernel_Name"])
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
    meta[k] = (r.get("Scratch_Size", ""), r.get("VGPR_Count", ""), r.get("Accum_VGPR_Count", ""))
flt = sys.argv[2:]
print(f"{'kernel':44s} {'disp':>5s} {'waves':>9s} {'VALU/wave':>11s} {'VALU/life%':>10s} {'LDS/wave':>9s} "
      f"{'scratch':>7s} {'vgpr':>5s}")
rows = sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_INSTS_VALU", 0))
for k, c in rows:
    if flt and not any(f in k for f in flt):
        continue
    w = max(c.get("SQ_WAVES", 0), 1)
    act = 100.0 * c.get("SQ_ACTIVE_INST_VALU", 0) / max(c.get("SQ_WAVE_CYCLES", 0), 1)
    sc, vg, ag = meta[k]
    print(f"{k[:44]:44s} {len(disp[k]):5d} {w:9.0f} {c.get('SQ_INSTS_VALU', 0) / w:11.0f} {act:10.1f} "
          f"{c.get('SQ_INSTS_LDS', 0) / w:9.1f} {sc:>7s} {vg:>5s}")
