"""``drynx-client``: network new|add-node|set-client ; survey new|set-operation|run
(reference cmd/client/main.go:33-69, network.go, survey.go:61-154).  Config
streams are TOML on stdin/stdout so commands pipe into each other."""
from __future__ import annotations

import argparse
import sys

from . import toml_io


def _read():
    data = sys.stdin.read() if not sys.stdin.isatty() else ""
    return toml_io.loads(data)


def _write(cfg):
    sys.stdout.write(toml_io.dumps(cfg))


def network_new(a):
    cfg = _read()
    cfg["Network"] = {"Nodes": []}
    _write(cfg)


def network_add_node(a):
    cfg = _read()
    net = cfg.setdefault("Network", {})
    net.setdefault("Nodes", []).append({"Address": a.address, "PublicKey": a.public})
    _write(cfg)


def network_set_client(a):
    cfg = _read()
    cfg.setdefault("Network", {})["Client"] = {"URL": a.address}
    _write(cfg)


def survey_new(a):
    cfg = _read()
    cfg["Survey"] = {"Name": a.name}
    _write(cfg)


def survey_set_operation(a):
    cfg = _read()
    cfg.setdefault("Survey", {})["Operation"] = a.operation
    _write(cfg)


def survey_run(a):
    """roster[0] is the CN (and the VN roster), roster[1:] are DPs; no proofs;
    GroupBy {3,2,1}; 10 rows in [0, 256] (survey.go:93-132)."""
    from ..crypto import oracle as O
    from ..query import QueryDPDataGen, QueryDiffP, Roster, ServerIdentity, choose_operation
    from ..services.api import DrynxClient
    from ..services.server import RemoteNode

    cfg = _read()
    nodes = cfg["Network"]["Nodes"]
    if len(nodes) < 2:
        raise SystemExit("need at least 2 nodes (1 CN + >=1 DP)")
    entry = cfg["Network"].get("Client", {}).get("URL") or nodes[0]["Address"]
    ids = [n["Address"] for n in nodes]
    pubs = {n["Address"]: O.g1_from_bytes(bytes.fromhex(n["PublicKey"])) for n in nodes}
    cn, dps = ids[0], ids[1:]
    roster = Roster([ServerIdentity(f"cn:{cn}", pubs[cn], cn, 0)])
    id_to_pub = {f"cn:{cn}": pubs[cn], f"vn:{cn}": pubs[cn]}
    id_to_pub.update({f"dp:{d}": pubs[d] for d in dps})
    s2dp = {f"cn:{cn}": [ServerIdentity(f"dp:{d}", pubs[d], d, i + 1) for i, d in enumerate(dps)]}
    op = choose_operation(cfg["Survey"]["Operation"], 0, 256, 5, 0)
    client = DrynxClient(RemoteNode(entry))  # the roster travels inside the SurveyQuery
    sq = client.generate_survey_query(roster, None, s2dp, id_to_pub, cfg["Survey"].get("Name"), op, None, None, 0,
                                      False, [0.0] * 5, QueryDiffP(), QueryDPDataGen([3, 2, 1], 10, 0, 256))
    groups, values, _ = client.send_survey_query(sq)
    first = values[0]
    if any(v != first for v in values):
        raise SystemExit(f"groups disagree: {values}")
    print(" ".join(str(v) for v in first))


def main(argv=None):
    ap = argparse.ArgumentParser(prog="drynx-client")
    sub = ap.add_subparsers(dest="group", required=True)
    net = sub.add_parser("network").add_subparsers(dest="cmd", required=True)
    net.add_parser("new").set_defaults(fn=network_new)
    p = net.add_parser("add-node")
    p.add_argument("address")
    p.add_argument("public")
    p.set_defaults(fn=network_add_node)
    p = net.add_parser("set-client")
    p.add_argument("address")
    p.set_defaults(fn=network_set_client)
    sv = sub.add_parser("survey").add_subparsers(dest="cmd", required=True)
    p = sv.add_parser("new")
    p.add_argument("name")
    p.set_defaults(fn=survey_new)
    p = sv.add_parser("set-operation")
    p.add_argument("operation")
    p.set_defaults(fn=survey_set_operation)
    sv.add_parser("run").set_defaults(fn=survey_run)
    a = ap.parse_args(argv)
    a.fn(a)
    return 0


if __name__ == "__main__":
    sys.exit(main())
