"""GPU time per framework span, from one rocprofv3 --runtime-trace run.

Run the bench with DRYNX_ROCTX=1 (every ``timers.span`` / ``timers.timed`` is
a roctx range) under ``rocprofv3 --runtime-trace --output-format csv -d D -o
run -- python bench.py ...``; then

    python tools/span_kernels.py D [--queries K] [--out file]

joins each kernel (kernel_trace: name, device duration) to the HIP call that
launched it (hip_api_trace: same Correlation_Id -> host thread and launch
time) and that call to the innermost roctx range open on its thread at that
moment (marker_api_trace).  Only kernels launched inside the last K
``bench.step`` ranges count (the timed queries; per-query averages).
Prints per span: kernel time, the part in non-hand-written kernels (torch /
ATen, rocPRIM, runtime copies and fills = "glue") and its largest glue
kernels -- the table behind the glue budget of profiles/r4/."""
from __future__ import annotations

import argparse
import bisect
import csv
import glob
import os
from collections import defaultdict


_SLOTS = 2048  # resident workgroups the chip can hold at once (256 CUs x 8)


def _find(d, suffix):
    got = sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True))
    if not got:
        raise SystemExit(f"no *{suffix} under {d}")
    return got[-1]


def _col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(names)


def glue(name: str) -> bool:
    return ("at::native" in name or "rocclr" in name or "rocprim" in name or "at::cuda" in name
            or "elementwise_kernel_with_index" in name or name.startswith("void (anonymous namespace)::elementwise"))


def short(name: str) -> str:
    for key, s in (("CatArrayBatchedCopy", "aten cat"), ("copyBuffer", "rocclr copyBuffer"),
                   ("fillBuffer", "rocclr fillBuffer"), ("direct_copy", "aten copy/convert"),
                   ("and_kernel", "aten all()"), ("onesweep", "rocprim sort"), ("index_elementwise", "aten index"),
                   ("scatter_gather", "aten gather/scatter"), ("reduce_kernel", "aten reduce"),
                   ("radixSort", "aten sort"), ("vectorized_elementwise", "aten elementwise"),
                   ("arange", "aten arange"), ("lookback_scan", "rocprim scan")):
        if key in name:
            return s
    n = name.split("(")[0]
    return n[-60:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--queries", type=int, default=3)
    ap.add_argument("--window", default="bench.step")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    # kernels by row (a Correlation_Id can repeat: several dispatches of one
    # call, and ids reused across threads)
    kern = {}
    iv = []
    with open(_find(a.dir, "kernel_trace.csv")) as f:
        for c, r in enumerate(csv.DictReader(f)):
            wgs = 1
            for ax in "XYZ":
                wgs *= max(1, int(r[f"Grid_Size_{ax}"]) // max(1, int(r[f"Workgroup_Size_{ax}"])))
            iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), c, min(wgs, _SLOTS)))
            kern[c] = [r["Kernel_Name"], 0.0, (int(r["Correlation_Id"]), r["Thread_Id"]), r["Thread_Id"],
                       int(r["Start_Timestamp"])]
    # kernels overlap (streams, and queue-level concurrency even under
    # AMD_SERIALIZE_KERNEL): each instant of device time is shared by the
    # kernels running then, in proportion to their workgroups (capped at the
    # chip's resident slots) -- a one-workgroup kernel beside a full-chip one
    # is charged ~nothing for the wait, not its whole stretched duration
    ev = sorted([(x[0], 1, i) for i, x in enumerate(iv)] + [(x[1], 0, i) for i, x in enumerate(iv)])
    srt = sorted(iv)
    overlaps = sum(1 for i in range(1, len(srt)) if srt[i][0] < max(x[1] for x in srt[max(0, i - 64): i]))
    raw = overlaps < 0.01 * max(1, len(iv))  # a serialized run: each kernel's own duration
    if raw:
        for s_, e_, c_, w_ in iv:
            kern[c_][1] = (e_ - s_) / 1e6
        ev = []
    active, wsum, last = set(), 0, None
    for t, kind, i in ev:
        if last is not None and active and t > last:
            dt = (t - last) / 1e6
            for j in active:
                kern[iv[j][2]][1] += dt * iv[j][3] / wsum
        last = t
        if kind == 1:
            active.add(i)
            wsum += iv[i][3]
        else:
            active.discard(i)
            wsum -= iv[i][3]
    from collections import Counter

    nkey = Counter(k[2] for k in kern.values())
    launch = {}
    with open(_find(a.dir, "hip_api_trace.csv")) as f:
        for r in csv.DictReader(f):
            key = (int(r["Correlation_Id"]), r["Thread_Id"])
            if key in nkey and key not in launch:
                launch[key] = (r["Thread_Id"], int(r["Start_Timestamp"]))
    ranges = defaultdict(list)  # thread -> [(start, end, name)]
    with open(_find(a.dir, "marker_api_trace.csv")) as f:
        for r in csv.DictReader(f):
            name = _col(r, "Function", "Message", "Name")
            ranges[r["Thread_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    for t in ranges:
        ranges[t].sort()
    wins = sorted((s, e) for rs in ranges.values() for s, e, n in rs if n == a.window)[-a.queries:]
    if not wins:
        raise SystemExit(f"no {a.window} ranges")
    starts = {t: [x[0] for x in rs] for t, rs in ranges.items()}

    def innermost(th, ts):
        rs = ranges.get(th, [])
        i = bisect.bisect_right(starts.get(th, []), ts)
        best = None
        for j in range(i - 1, max(-1, i - 400), -1):
            s, e, n = rs[j]
            if s <= ts <= e and (best is None or s > best[0]):
                best = (s, e, n)
                break
        return best[2] if best else "(no span)"

    tot = defaultdict(float)
    gl = defaultdict(float)
    cnt = defaultdict(int)
    gk = defaultdict(lambda: defaultdict(float))
    all_k = all_g = 0.0
    for c, (name, dur, key, kth, kstart) in kern.items():
        # the launching call's time; for an ambiguous id the kernel's own start
        # (a serialized run starts each kernel right after its launch)
        th, ts = launch[key] if (key in launch and nkey[key] == 1) else (kth, kstart)
        if not any(s <= ts <= e for s, e in wins):
            continue
        sp = innermost(th, ts)
        tot[sp] += dur
        cnt[sp] += 1
        all_k += dur
        if glue(name):
            gl[sp] += dur
            all_g += dur
            gk[sp][short(name)] += dur
    q = len(wins)
    # wall and device-busy time of the windows (union of kernel intervals inside them)
    wall = sum(e - s_ for s_, e in wins) / 1e6 / q
    busy = 0
    for ws, we in wins:
        segs = sorted((max(x[0], ws), min(x[1], we)) for x in iv if x[1] > ws and x[0] < we)
        cur_s = cur_e = None
        for s_, e in segs:
            if cur_e is None or s_ > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s_, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            busy += cur_e - cur_s
    busy = busy / 1e6 / q
    lines = [f"# kernels launched inside the last {q} '{a.window}' ranges, per query (ms of device time, "
             + ("serialized run: each kernel's own duration)" if raw else
                f"{overlaps} overlapping kernels: overlap shared by workgroups)"),
             f"# all kernels {all_k / q:.2f} ms, glue (torch/ATen, rocPRIM, runtime copies/fills) {all_g / q:.2f} ms",
             f"# window wall {wall:.2f} ms, device busy {busy:.2f} ms ({100 * busy / max(wall, 1e-9):.0f}%)",
             f"{'span':40s} {'kernel_ms':>9s} {'glue_ms':>8s} {'n':>6s}  largest glue kernels"]
    for sp in sorted(tot, key=lambda k: -tot[k]):
        top = ", ".join(f"{k} {v / q:.2f}" for k, v in sorted(gk[sp].items(), key=lambda kv: -kv[1])[:3])
        lines.append(f"{sp[:40]:40s} {tot[sp] / q:9.2f} {gl[sp] / q:8.2f} {cnt[sp] / q:6.0f}  {top}")
    txt = "\n".join(lines) + "\n"
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()
