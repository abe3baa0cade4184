"""``drynx-server``: gen | run  (reference cmd/server/main.go:42-131).

  python -m drynx_amd.cli.server gen host:node-port host:client-port > node.toml
  python -m drynx_amd.cli.server run < node.toml
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
    r = sub.add_parser("run", help="read the node config on stdin and serve")
    r.add_argument("--workdir", default=None)
    r.add_argument("--device", default=None)
    r.add_argument("--group", default=None,
                   help="group file: a TOML network config ([[Network.Nodes]] Address/PublicKey) listing the nodes "
                        "this node may form a cluster with")
    r.add_argument("--trust-any", action="store_true", help="accept a join from any root (local experiments)")
    a = ap.parse_args(argv)
    from ..services import server as srv

    if a.cmd == "gen":
        cfg = srv.gen_config(a.node_address, a.client_address, a.description)
        sys.stdout.write(toml_io.dumps({"Server": cfg}))
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
