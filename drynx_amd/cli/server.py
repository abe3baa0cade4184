"""``drynx-server``: gen | run  (reference cmd/server/main.go:42-131), plus
the role filters its README documents (cmd/README.md:20-35; the reference's
binary has only gen and run):

  python -m drynx_amd.cli.server new host:node-port host:client-port |
      python -m drynx_amd.cli.server data-provider new file-loader records.csv |
      python -m drynx_amd.cli.server computing-node new |
      python -m drynx_amd.cli.server verifying-node new > node.toml
  python -m drynx_amd.cli.server run < node.toml

``new`` is ``gen``.  A role filter reads the config stream on stdin and adds
its section: a node whose config has role sections serves only those roles
(a survey that gives it another role is refused); a config without any serves
every role.  A data provider with a file loader answers from its file
(``models.datasets.load_dp_file``) instead of the query's generated data.
"""
from __future__ import annotations

import argparse
import sys

from . import toml_io


def main(argv=None):
    ap = argparse.ArgumentParser(prog="drynx-server")
    sub = ap.add_subparsers(dest="cmd", required=True)
    g = sub.add_parser("gen", help="generate a new node keypair + config on stdout")
    g.add_argument("node_address")
    g.add_argument("client_address", nargs="?", default="")
    g.add_argument("--description", default="")
    n = sub.add_parser("new", help="same as gen")
    n.add_argument("node_address")
    n.add_argument("client_address", nargs="?", default="")
    n.add_argument("--description", default="")
    dp = sub.add_parser("data-provider", help="config filter: serve the data-provider role")
    dp_sub = dp.add_subparsers(dest="dp_cmd", required=True)
    dpn = dp_sub.add_parser("new", help="add the DataProvider section")
    dpn_sub = dpn.add_subparsers(dest="source", required=True)
    fl = dpn_sub.add_parser("file-loader", help="answer from a file of records (comma-separated)")
    fl.add_argument("path")
    for role in ("computing-node", "verifying-node"):
        rp_ = sub.add_parser(role, help=f"config filter: serve the {role} role")
        rp_.add_subparsers(dest=role.replace("-", "_") + "_cmd", required=True).add_parser(
            "new", help=f"add the {role} section")
    r = sub.add_parser("run", help="read the node config on stdin and serve")
    r.add_argument("--workdir", default=None)
    r.add_argument("--device", default=None)
    r.add_argument("--group", default=None,
                   help="group file: a TOML network config ([[Network.Nodes]] Address/PublicKey) listing the nodes "
                        "this node may form a cluster with")
    r.add_argument("--trust-any", action="store_true", help="accept a join from any root (local experiments)")
    a = ap.parse_args(argv)
    from ..services import server as srv

    if a.cmd in ("gen", "new"):
        cfg = srv.gen_config(a.node_address, a.client_address, a.description)
        sys.stdout.write(toml_io.dumps({"Server": cfg}))
        return 0
    if a.cmd in ("data-provider", "computing-node", "verifying-node"):
        doc = toml_io.loads(sys.stdin.read())
        cfg = doc["Server"]
        if a.cmd == "data-provider":
            import os

            cfg["DataProvider"] = {"Source": "file-loader", "Path": os.path.abspath(a.path)}
        else:
            cfg["ComputingNode" if a.cmd == "computing-node" else "VerifyingNode"] = {"Enabled": True}
        sys.stdout.write(toml_io.dumps(doc))
        return 0
    cfg = toml_io.loads(sys.stdin.read())["Server"]
    if a.group:
        with open(a.group) as f:
            group = toml_io.loads(f.read())
        cfg["Trusted"] = [n["PublicKey"] for n in group.get("Network", {}).get("Nodes", [])]
    cfg["TrustAny"] = bool(a.trust_any)
    from ..utils.streams import node_process_setup

    node_process_setup()
    srv.NodeServer(cfg, a.workdir, a.device).serve_forever()
    return 0


if __name__ == "__main__":
    sys.exit(main())
