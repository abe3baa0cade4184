"""Benchmark plots from the measured logs in ``profiles/`` (the role of the
reference's ``simul/test_data/graphs/TIFS/*.py`` scripts, A34 in SURVEY.md:
allOps.py, diffPri.py, logReg*.py, timeline.py).  Those scripts hard-code
numbers measured on a CPU cluster; these read this framework's JSON-lines
logs, which already carry the reference value for every row (AllResults.xlsx
sheets AllOps / DiffPri / LogReg, quoted in BASELINE.md), and draw both.

    python tools/plot_results.py [--profiles profiles] [--out profiles/plots] [--fmt pdf]

Outputs: allops.<fmt> (per-operation query time, log scale), scaling.<fmt>
(ScaleServers / ScaleVNs sweeps), dro.<fmt>
(shuffle prove/verify vs noise-list size), lr_timeline.<fmt> (phases of the
headline verifiable LR query from the bench line's ``phase_s``), and
summary.csv with the plotted numbers.
"""
from __future__ import annotations

import argparse
import csv
import json
import os

# DiffPri sheet (whole query with a noise list of this size), BASELINE.md / SURVEY.md §6
REF_DRO_QUERY_S = {10_000: 82.0, 100_000: 657.0, 1_000_000: 5872.0}
REF_LR_SPECTF_S = 196.77


def _jsonl(path: str) -> list:
    out = []
    if not os.path.exists(path):
        return out
    with open(path) as f:
        for line in f:
            line = line.strip()
            if line.startswith("{"):
                try:
                    out.append(json.loads(line))
                except json.JSONDecodeError:
                    pass
    return out


def load(profiles: str) -> dict:
    allops = [r for r in _jsonl(os.path.join(profiles, "r1_bench_allops_1gpu.log")) if "op" in r]
    dro = [r for r in _jsonl(os.path.join(profiles, "r1_bench_dro_shuffle_1gpu.log")) if "n" in r]
    bench = [r for r in _jsonl(os.path.join(profiles, "r1_bench_final_1gpu.log")) if "metric" in r]
    scaling = [r for r in _jsonl(os.path.join(profiles, "r1_bench_scaling_1gpu.log")) if "sweep" in r]
    return {"allops": allops, "dro": dro, "bench": bench[-1] if bench else None, "scaling": scaling}


def write_summary(data: dict, path: str):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["benchmark", "item", "this_s", "reference_s", "speedup"])
        for r in data["allops"]:
            w.writerow(["allops", r["op"], r["seconds"], r["reference_s"], r["speedup"]])
        for r in data["dro"]:
            ref = REF_DRO_QUERY_S.get(r["n"])
            tot = r["shuffle_prove_s"] + r["verify_s"]
            # the reference number is a whole query with that noise list, not the
            # shuffle alone: no speed-up is claimed for these rows
            w.writerow(["dro_shuffle_prove_plus_verify", r["n"], round(tot, 4), ref, ""])
        for r in data.get("scaling", []):
            w.writerow([r["sweep"], f"{r['cns']} CNs / {r['dps']} DPs / {r['vns']} VNs", r["seconds"],
                        r["reference_s"] or "", r["speedup"] or ""])
        b = data["bench"]
        if b is not None:
            w.writerow(["lr_query", b["config"]["model"], b["e2e_latency_s"], REF_LR_SPECTF_S,
                        round(REF_LR_SPECTF_S / b["e2e_latency_s"], 1)])


def plot(data: dict, out: str, fmt: str):
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    made = []
    if data["allops"]:
        ops = [r["op"] for r in data["allops"]]
        fig, ax = plt.subplots(figsize=(10, 4.5))
        x = range(len(ops))
        ax.bar([i - 0.2 for i in x], [r["reference_s"] for r in data["allops"]], 0.4, label="reference (CPU cluster)")
        ax.bar([i + 0.2 for i in x], [r["seconds"] for r in data["allops"]], 0.4, label="drynx_amd (1 MI355X)")
        ax.set_yscale("log")
        ax.set_ylabel("verifiable query time (s)")
        ax.set_xticks(list(x))
        ax.set_xticklabels(ops, rotation=35, ha="right", fontsize=8)
        ax.legend()
        fig.tight_layout()
        p = os.path.join(out, f"allops.{fmt}")
        fig.savefig(p)
        plt.close(fig)
        made.append(p)
    if data["dro"]:
        ns = [r["n"] for r in data["dro"]]
        fig, ax = plt.subplots(figsize=(6, 4))
        ax.plot(ns, [r["shuffle_prove_s"] for r in data["dro"]], "o-", label="shuffle + proof (1 CN)")
        ax.plot(ns, [r["verify_s"] for r in data["dro"]], "s-", label="proof verification (1 VN)")
        ref = [(n, REF_DRO_QUERY_S[n]) for n in ns if n in REF_DRO_QUERY_S]
        if ref:
            ax.plot([a for a, _ in ref], [b for _, b in ref], "k--", label="reference: whole query")
        ax.set_xscale("log")
        ax.set_yscale("log")
        ax.set_xlabel("noise-list size")
        ax.set_ylabel("seconds")
        ax.legend()
        fig.tight_layout()
        p = os.path.join(out, f"dro.{fmt}")
        fig.savefig(p)
        plt.close(fig)
        made.append(p)
    sc = data.get("scaling", [])
    if sc:
        fig, axes = plt.subplots(1, 2, figsize=(10, 4))
        for ax, key, xname in ((axes[0], "ScaleServers", "cns"), (axes[1], "ScaleVNs", "vns")):
            for sweep in dict.fromkeys(r["sweep"] for r in sc if r["sweep"].startswith(key)):
                pts = [r for r in sc if r["sweep"] == sweep]
                ax.plot([r[xname] for r in pts], [r["seconds"] for r in pts], "o-", label=f"drynx_amd: {sweep}")
                ref = [r for r in pts if r["reference_s"]]
                ax.plot([r[xname] for r in ref], [r["reference_s"] for r in ref], "x--", label=f"reference: {sweep}")
            ax.set_yscale("log")
            ax.set_xlabel("#" + xname.upper())
            ax.set_ylabel("seconds per verifiable sum query")
            ax.legend(fontsize=7)
        fig.tight_layout()
        p = os.path.join(out, f"scaling.{fmt}")
        fig.savefig(p)
        plt.close(fig)
        made.append(p)
    b = data["bench"]
    if b is not None and b.get("phase_s"):
        keep = ["dp0_DPencoding", "cn0_AggregationPhase", "KeySwitchingPhase", "JustExecution", "Decode",
                "vn0_VerifyRange", "vn0_VerifyKeySwitch", "ProofVerification", "BI"]
        ph = [(k, b["phase_s"][k]) for k in keep if k in b["phase_s"]]
        fig, ax = plt.subplots(figsize=(7, 4))
        ax.barh([k for k, _ in ph][::-1], [v * 1e3 for _, v in ph][::-1])
        ax.set_xlabel("ms (phases overlap; see profiles/r1_host_trace_1gpu.txt)")
        ax.set_title(f"verifiable LR query: {b['e2e_latency_s'] * 1e3:.1f} ms end to end "
                     f"(reference LR SPECTF {REF_LR_SPECTF_S} s)", fontsize=9)
        fig.tight_layout()
        p = os.path.join(out, f"lr_timeline.{fmt}")
        fig.savefig(p)
        plt.close(fig)
        made.append(p)
    return made


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--profiles", default="profiles")
    ap.add_argument("--out", default=os.path.join("profiles", "plots"))
    ap.add_argument("--fmt", default="pdf", choices=["pdf", "png", "svg"])
    a = ap.parse_args(argv)
    os.makedirs(a.out, exist_ok=True)
    data = load(a.profiles)
    write_summary(data, os.path.join(a.out, "summary.csv"))
    for p in plot(data, a.out, a.fmt):
        print(p)


if __name__ == "__main__":
    main()
