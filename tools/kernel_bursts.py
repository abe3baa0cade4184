#!/usr/bin/env python3
"""Per-kernel GPU time of the bursts of a rocprofv3 kernel trace (CSV):
bursts are runs of kernels separated by idle gaps longer than --gap ms (a
tool that wants a code path measured alone sleeps around it, e.g.
tools/rank_share.py).  Prints the last --last bursts, each with its kernels
by total time.  Usage: kernel_bursts.py trace.csv [--gap 300] [--last 2]"""
import argparse
import csv
from collections import defaultdict


def _name(n: str) -> str:
    if n.startswith("(anonymous namespace)::"):
        n = n[len("(anonymous namespace)::"):]
    if "for_each_kernel" in n and "<" in n:
        return n.split("<", 1)[1].split("::")[0]
    return n.split("(")[0][:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap", type=float, default=300.0)
    ap.add_argument("--last", type=int, default=2)
    a = ap.parse_args()
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in csv.DictReader(open(a.trace)))
    bursts, cur, end = [], [], None
    for s, e, n in iv:
        if end is not None and s - end > a.gap * 1e6:
            bursts.append(cur)
            cur = []
        cur.append((s, e, n))
        end = e if end is None else max(end, e)
    bursts.append(cur)
    for b in bursts[-a.last:]:
        agg = defaultdict(lambda: [0, 0.0])
        for s, e, n in b:
            x = agg[_name(n)]
            x[0] += 1
            x[1] += (e - s) / 1e6
        span = (max(e for _, e, _ in b) - b[0][0]) / 1e6
        print(f"burst: {len(b)} kernels, {sum(v[1] for v in agg.values()):.2f} ms of kernel time, {span:.2f} ms wall")
        for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
            print(f"  {v[1]:8.2f} ms {v[0]:5d}  {k}")


if __name__ == "__main__":
    main()
