#!/usr/bin/env python3
"""Timeline of one burst of a rocprofv3 kernel trace (CSV): every kernel of
the burst (bursts: runs separated by idle gaps > --gap ms, as
tools/kernel_bursts.py) with its start / end offset in ms, its queue and its
duration, plus the union busy time -- shows which kernels overlap and where
the device idles.  Usage: kernel_timeline.py trace.csv [--gap 300] [--burst -1] [--min-ms 0.05]"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap", type=float, default=300.0)
    ap.add_argument("--burst", type=int, default=-1)
    ap.add_argument("--min-ms", type=float, default=0.05)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    qkey = next((k for k in ("Queue_Id", "Stream_Id", "Dispatch_Id") if k in rows[0]), None)
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get(qkey, "?")) for r in rows)
    bursts, cur, end = [], [], None
    for s, e, n, q in iv:
        if end is not None and s - end > a.gap * 1e6:
            bursts.append(cur)
            cur = []
        cur.append((s, e, n, q))
        end = e if end is None else max(end, e)
    bursts.append(cur)
    b = bursts[a.burst]
    t0 = b[0][0]
    busy, last = 0, t0
    for s, e, _, _ in b:
        if e > last:
            busy += e - max(s, last)
            last = e
    span = max(e for _, e, _, _ in b) - t0
    print(f"burst: {len(b)} kernels, wall {span / 1e6:.2f} ms, device busy (union) {busy / 1e6:.2f} ms")
    for s, e, n, q in b:
        if (e - s) / 1e6 >= a.min_ms:
            nm = n.replace("(anonymous namespace)::", "").split("(")[0][:60]
            print(f"{(s - t0) / 1e6:8.2f} {(e - t0) / 1e6:8.2f} {(e - s) / 1e6:7.2f}  q{q:<4} {nm}")


if __name__ == "__main__":
    main()
