"""Print the kernel timeline of the last bench step from a rocprofv3 kernel trace."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "dx_elgamal_encrypt" in r["Kernel_Name"]]
last = rows[starts[-1]:]
t0 = int(last[0]["Start_Timestamp"])
prev_end = t0
agg = []
for r in last:
    nm = r["Kernel_Name"]
    nm = nm.split("<")[1].split("::")[0] if "<" in nm else nm.split("(")[0][:40]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    agg.append((nm, (s - t0) / 1e6, (e - s) / 1e6, (s - prev_end) / 1e6, r["Grid_Size_X"]))
    prev_end = e
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3
print(f"step wall {(prev_end - t0) / 1e6:.1f} ms, kernels {len(agg)}, busy {sum(a[2] for a in agg):.1f} ms")
for nm, st, d, gap, grid in agg:
    if d > thr or gap > 2:
        print(f"t={st:8.2f} dur={d:7.2f} gap={gap:6.2f} grid={grid:>8} {nm}")
