"""Static register / scratch / occupancy table of every gfx950 kernel.

Compiles each ``csrc/kernels/*.hip`` device side only (``--cuda-device-only``)
with ``-Rpass-analysis=kernel-resource-usage`` and tabulates, per kernel, the
compiler's VGPRs / AGPRs / SGPRs, scratch bytes per lane (spills and private
arrays) and waves per SIMD.  This is the compile-time counterpart of the
PMC scratch column (``tools/pmc_summary.py``): a kernel listed here with
scratch 0 cannot spill at run time.

Usage: python tools/kernel_resources.py [--only name,...] [--filter substr] [-j 8] > table.txt
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KDIR = os.path.join(ROOT, "csrc", "kernels")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FIELDS = {"VGPRs": "vgpr", "AGPRs": "agpr", "SGPRs": "sgpr", "ScratchSize [bytes/lane]": "scratch",
          "Occupancy [waves/SIMD]": "occ", "LDS Size [bytes/block]": "lds"}


def _demangle(names):
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                           text=True, timeout=60)
        out = r.stdout.splitlines()
        if len(out) == len(names):
            return out
    except (OSError, subprocess.SubprocessError):
        pass
    return names


EXTRA: list[str] = []


def analyse(src: str) -> list[dict]:
    with tempfile.TemporaryDirectory() as td:
        cmd = [HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only", "-I",
               os.path.join(ROOT, "csrc"), "-c", src, "-o", os.path.join(td, "k.o"),
               "-Rpass-analysis=kernel-resource-usage", *EXTRA]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=1800)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: (?:\s*)(.+?): (.+?) \[-Rpass-analysis", line)
        if not m:
            continue
        key, val = m.group(1).strip(), m.group(2).strip()
        if key == "Function Name":
            cur = {"tu": os.path.basename(src), "name": val}
            rows.append(cur)
        elif cur is not None and key in FIELDS:
            try:
                cur[FIELDS[key]] = int(val)
            except ValueError:
                cur[FIELDS[key]] = val
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None, help="comma list of TU basenames (no extension)")
    ap.add_argument("--filter", default=None, help="keep kernels whose demangled name contains this")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("-D", action="append", default=[], help="extra preprocessor define (e.g. DX_OCC_WAVES=1)")
    a = ap.parse_args()
    EXTRA.extend(f"-D{d}" for d in a.D)
    srcs = sorted(os.path.join(KDIR, f) for f in os.listdir(KDIR) if f.endswith(".hip"))
    if a.only:
        keep = set(a.only.split(","))
        srcs = [s for s in srcs if os.path.splitext(os.path.basename(s))[0] in keep]
    with cf.ThreadPoolExecutor(a.j) as ex:
        rows = [r for rs in ex.map(analyse, srcs) for r in rs]
    names = _demangle([r["name"] for r in rows])
    seen = set()
    print(f"{'scratch':>7} {'vgpr':>4} {'agpr':>4} {'occ':>3} {'lds':>6}  {'tu':18s} kernel")
    for r, n in sorted(zip(rows, names), key=lambda rn: (-rn[0].get("scratch", 0), rn[1])):
        # the host-callable for_each_kernel / for_each_kernel64 twins of one lambda: keep the 64-lane one
        short = n.replace("(anonymous namespace)::", "")
        m = re.match(r"void dx::for_each_kernel(?:64)?<(\w+)::\{lambda\(long\)#(\d+)\}>", short)
        short = f"{m.group(1)}#{m.group(2)}" if m else re.sub(r"^void ", "", re.sub(r"\(.*$", "", short))
        if a.filter and a.filter not in short:
            continue
        key = (r["tu"], short)
        if key in seen:
            continue
        seen.add(key)
        print(f"{r.get('scratch', 0):7d} {r.get('vgpr', 0):4d} {r.get('agpr', 0):4d} {r.get('occ', 0):3d} "
              f"{r.get('lds', 0):6d}  {r['tu']:18s} {short[:110]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
