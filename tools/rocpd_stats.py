"""Per-kernel statistics from a rocprofv3 SQLite (rocpd) database: total /
count / mean time per kernel name, sorted by total; optional time window
(the last N ms of the trace).  Usage: python tools/rocpd_stats.py db [top] [last_ms]"""
import collections
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    last_ms = float(sys.argv[3]) if len(sys.argv) > 3 else None
    names = {r[0]: (r[1], r[2], r[3], r[4]) for r in db.execute(
        "select id, display_name, arch_vgpr_count, accum_vgpr_count, private_segment_size "
        "from rocpd_info_kernel_symbol")}
    agg = collections.defaultdict(lambda: [0, 0.0])
    t_min, t_max = None, None
    rows = db.execute("select kernel_id, start, end from rocpd_kernel_dispatch").fetchall()
    if last_ms is not None and rows:
        t_end = max(r[2] for r in rows)
        rows = [r for r in rows if r[1] >= t_end - last_ms * 1e6]
    for kid, s, e in rows:
        a = agg[kid]
        a[0] += 1
        a[1] += (e - s) / 1e6
        t_min = s if t_min is None else min(t_min, s)
        t_max = e if t_max is None else max(t_max, e)
    tot = sum(v[1] for v in agg.values())
    print(f"kernels: {sum(v[0] for v in agg.values())} dispatches, {tot:.1f} ms busy, "
          f"span {(t_max - t_min) / 1e6:.1f} ms")
    print(f"{'ms':>9} {'n':>6} {'mean_us':>9} {'vgpr':>5} {'agpr':>5} {'scratch':>7}  kernel")
    for kid, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        nm, vg, ag, sc = names.get(kid, ("?", 0, 0, 0))
        nm = nm if len(nm) < 90 else nm[:87] + "..."
        print(f"{ms:9.2f} {n:6d} {1000 * ms / n:9.1f} {vg:5d} {ag:5d} {sc:7d}  {nm}")


if __name__ == "__main__":
    main()
