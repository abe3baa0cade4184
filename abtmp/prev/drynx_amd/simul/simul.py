"""Simulation harness (reference simul/drynx_simul.go + simul/runfiles/*.toml).

Reads an onet-style runfile — global ``key = value`` lines followed by a
CSV-like table whose header names the per-run parameters (Hosts, NbrServers,
NbrVNs, NbrDPs, NbrDPsPerServer, Proofs, Ranges, Obfuscation, OperationName,
NbrInput, NbrOutput, DiffP*, DPRows, MinData, MaxData, ThresholdGeneral,
ThresholdOther, CuttingFactor, NbrRecords, MaxIterations) — and runs every
row ``Rounds`` times through the framework, recording the reference's named
timers into a CSV (``Simulation`` wraps each run).

Usage: python -m drynx_amd.simul.simul drynx_amd/simul/runfiles/drynx.toml [--csv out.csv]
(multi-GPU: under torch.distributed.run, parties are spread over the ranks.)
"""
from __future__ import annotations

import argparse
import ast
import csv
import sys
import tempfile

from ..parallel.comm import init_distributed, make_comm
from ..parallel.netem import flow_hops
from ..query import QueryDiffP, LogisticRegressionParameters
from ..services.api import DrynxClient
from ..services.local import local_cluster, make_survey
from ..utils import timers
from ..utils.log import get_logger

log = get_logger("simul")


def parse_runfile(text: str):
    glob, header, rows = {}, None, []
    for raw in text.splitlines():
        line = raw.strip()
        if not line or line.startswith("#"):
            continue
        if header is None and "=" in line and "," not in line.split("=")[0]:
            k, v = line.split("=", 1)
            v = v.strip()
            lit = {"true": "True", "false": "False"}.get(v, v)
            try:
                glob[k.strip()] = ast.literal_eval(lit)
            except (ValueError, SyntaxError):
                glob[k.strip()] = v.strip('"')
            continue
        parts = [p.strip() for p in next(csv.reader([line], skipinitialspace=True))]
        if header is None:
            header = parts
        else:
            row = {}
            for k, v in zip(header, parts):
                vv = v.strip().strip('"')
                if vv.lower() in ("true", "false"):
                    row[k] = vv.lower() == "true"
                else:
                    try:
                        row[k] = int(vv)
                    except ValueError:
                        try:
                            row[k] = float(vv)
                        except ValueError:
                            row[k] = vv
            rows.append(row)
    return glob, rows


def ranges_for(code: int, n_out: int):
    """simul/drynx_simul.go:133-281 `Ranges` presets."""
    presets = {0: (0, 0), 1: (2, 1), 16: (16, 16), 17: (8, 3), 18: (16, 5), 19: (4, 16)}
    if code == -1:
        return None
    if code in presets:
        return [list(presets[code]) for _ in range(n_out)]
    if 99 <= code <= 103:  # per-output mixes used for variance (sum, N, sum of squares)
        mix = {99: [(16, 4), (16, 2), (16, 8)], 100: [(16, 5), (16, 3), (16, 10)], 101: [(16, 6), (16, 4), (16, 12)],
               102: [(16, 8), (16, 5), (16, 16)], 103: [(16, 16), (16, 16), (16, 16)]}[code]
        return [list(mix[i % len(mix)]) for i in range(n_out)]
    raise ValueError(f"unknown Ranges preset {code}")


def run_row(glob: dict, row: dict, comm, device, workdir, netem: str = "sleep"):
    n_cn, n_vn, n_dp = int(row["NbrServers"]), int(row.get("NbrVNs", 0)), int(row["NbrDPs"])
    proofs = int(row.get("Proofs", 0))
    if proofs and n_vn == 0:
        n_vn = 1
    cl, node = local_cluster(n_cn, n_dp, max(n_vn, 1), comm=comm, device=device, workdir=workdir)
    # the runfile's emulated links (drynx.toml:6-7): per-row Bandwidth / Delay
    # columns override the global keys (the reference's Bandwith sheet sweeps them)
    bw, dl = row.get("Bandwidth", glob.get("Bandwidth")), row.get("Delay", glob.get("Delay"))
    if netem != "off" and bw and dl is not None:
        from ..parallel.netem import NetEmulator

        node.net = NetEmulator(float(bw), float(dl), netem)
    # NbrDPsPerServer: the first CNs get that many DPs each (drynx_simul.go:317-333)
    per = int(row.get("NbrDPsPerServer", 0)) or max(1, n_dp // n_cn)
    op_name = str(row["OperationName"])
    lr = None
    d = int(row.get("NbrInput", 1)) - 1 if op_name == "lin_reg" else 1
    if op_name == "logistic regression":
        n_feat = int(glob.get("NbrFeatures", row.get("NbrInput", 8)))
        lr = LogisticRegressionParameters(NbrRecords=int(row.get("NbrRecords", 100)), NbrFeatures=n_feat,
                                          Lambda=1.0, Step=0.012, MaxIterations=int(row.get("MaxIterations", 25)),
                                          InitialWeights=[0.1] * (n_feat + 1), K=2,
                                          PrecisionApproxCoefficients=100.0, Means=[1.5] * n_feat,
                                          StandardDeviations=[1.1] * n_feat)
    diffp = None
    if int(row.get("DiffPSize", 0)):
        diffp = QueryDiffP(LapMean=float(row.get("DiffPEpsilon", 0)),
                           LapScale=max(1e-3, float(row.get("DiffPDelta", 1))),
                           NoiseListSize=int(row["DiffPSize"]), Quanta=float(row.get("DiffPQuanta", 1)),
                           Scale=float(row.get("DiffPScale", 1)), Limit=float(row.get("DiffPLimit", 1)))
    results = []
    client = DrynxClient(node, device=device) if comm.rank == 0 else None
    for rnd in range(int(glob.get("Rounds", 1))):
        t = timers.start_timer("Simulation")
        if comm.rank == 0:
            from ..query import choose_operation

            n_out = lr and 0 or choose_operation(op_name, int(row.get("MinData", 0)), int(row.get("MaxData", 1)), d,
                                                 int(row.get("CuttingFactor", 0))).NbrOutput
            if lr is not None:
                from ..query import lr_nbr_outputs

                n_out = lr_nbr_outputs(lr.NbrFeatures, lr.K)
            rg = ranges_for(int(row.get("Ranges", -1)), n_out) if proofs else None
            thr_g, thr_o = float(row.get("ThresholdGeneral", 0)), float(row.get("ThresholdOther", 0))
            obf = bool(row.get("Obfuscation", False))
            sq = make_survey(client, cl, op_name, query_min=int(row.get("MinData", 0)),
                             query_max=int(row.get("MaxData", 1)), d=d, rows=int(row.get("DPRows", 1)),
                             group_by=glob.get("GroupByValues", [1]), proofs=proofs, ranges=rg, obfuscation=obf,
                             thresholds=[thr_g, thr_o, thr_o, thr_o if obf else 0.0, thr_o] if proofs else None,
                             diffp=diffp, cutting_factor=int(row.get("CuttingFactor", 0)), lr_params=lr,
                             sig_device=device)
            # repartition DPs to CNs
            ids = [p.identity() for p in cl.dps]
            sq.ServerToDP = {c.id: ids[i * per:(i + 1) * per] for i, c in enumerate(cl.cns)}
            rest = ids[n_cn * per:]
            if rest:
                sq.ServerToDP[cl.cns[0].id] += rest
            net = node.net
            vn_ids = [v.id for v in cl.vns]
            if net is not None and proofs:
                # the simulation client hands the query to every VN first (drynx_simul.go:382-393)
                net.step("query_vns", [("client", v, 4096) for v in vn_ids], hops=flow_hops("query_vns", n_vns=n_vn))
            _, vals, res = client.send_survey_query(sq)
            results.append(vals[0])
            if net is not None and proofs:
                # CloseDB at every VN, then GetLatestBlock (drynx_simul.go:427-446)
                net.step("close_db", [("client", v, 64) for v in vn_ids], hops=flow_hops("close_db", n_vns=n_vn))
                net.step("latest_block", [("client", vn_ids[0], 1024), (vn_ids[0], "client", 4096)],
                         hops=flow_hops("latest_block"))
        else:
            node.run_survey(None)
        timers.end_timer(t)
    node.close(remove=True)
    return results


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("runfile")
    ap.add_argument("--csv", default=None)
    ap.add_argument("--device", default=None)
    ap.add_argument("--netem", default="sleep", choices=["sleep", "account", "off"],
                    help="apply the runfile's Bandwidth/Delay: wait where messages flow (sleep), only "
                         "record them (account), or ignore them (off)")
    a = ap.parse_args(argv)
    init_distributed()
    comm = make_comm(a.device)
    glob, rows = parse_runfile(open(a.runfile).read())
    out_rows = []
    for i, row in enumerate(rows):
        timers.reset()
        with tempfile.TemporaryDirectory() as wd:
            res = run_row(glob, row, comm, comm.device, wd, a.netem)
        summ = timers.summary()
        timers.dump_trace()  # DRYNX_TRACE=<path>: host span trace of the runs
        if comm.rank == 0:
            net = summ.get("NetworkEmulated", {}).get("sum", 0.0) / max(1, int(glob.get("Rounds", 1)))
            log.info(f"row {i}: {row.get('OperationName')} -> {res[-1] if res else None} "
                     f"(Simulation {summ['Simulation']['mean']:.3f}s, of which emulated network {net:.3f}s)")
            rounds = max(1, int(glob.get("Rounds", 1)))
            # timers recorded once per run: the mean; network steps: their total per run
            out_rows.append({"row": i, **{k: (v["sum"] / rounds if k.startswith(("net_", "NetworkEmulated"))
                                              else v["mean"]) for k, v in summ.items()}})
    if comm.rank == 0 and a.csv:
        keys = sorted({k for r in out_rows for k in r})
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=keys)
            w.writeheader()
            w.writerows(out_rows)
    return 0


def parse_time_data(path: str, flags=None) -> dict:
    """simul/test_data/parse_time_data_test.go: CSV with named timers -> table."""
    with open(path) as f:
        rows = list(csv.DictReader(f))
    out = {}
    for r in rows:
        for k, v in r.items():
            if flags and not any(fl in k for fl in flags):
                continue
            try:
                out.setdefault(k, []).append(float(v))
            except (TypeError, ValueError):
                pass
    return out


if __name__ == "__main__":
    sys.exit(main())
