"""Summarise a DRYNX_TRACE host span trace: per-thread timeline of the last
step (spans > threshold ms) and totals per span name."""
import json
import sys
from collections import defaultdict

ev = json.load(open(sys.argv[1]))["traceEvents"]
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
steps = [e for e in ev if e["name"] == "JustExecution"]
t0 = steps[-1]["ts"] if steps else min(e["ts"] for e in ev)
last = sorted((e for e in ev if e["ts"] >= t0 - 1), key=lambda e: e["ts"])
tot = defaultdict(float)
for e in last:
    tot[e["name"]] += e["dur"] / 1e3
    if e["dur"] / 1e3 >= thr:
        print(f"{(e['ts'] - t0) / 1e3:8.2f} +{e['dur'] / 1e3:7.2f} ms  [{e['tid'][:18]:18s}] {e['name']}")
print("--- totals (last step)")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:40]:
    print(f"{v:8.2f} ms  {k}")
