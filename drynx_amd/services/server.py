"""Standalone node servers + TCP control plane (the onet ``Server`` equivalent).

Reference: cmd/server/main.go (``gen`` keypair + config, ``run`` reads the
config and serves), the websocket client API (services/api.go:42), and the
multi-process test of test/lib.sh (3 real servers on localhost).

Model: every ``server run`` process is one node (one GPU or one CPU worker)
with its own long-term key.  A client sends a survey (with the roster it
chose, cmd/client/survey.go:93-132) to an entry node.  On the first survey the
entry node becomes rank 0 of a torch.distributed group it rendezvouses with
the roster nodes (``join`` message: world size, rank, master address); RCCL is
used when every node has a GPU, gloo otherwise.  All later surveys reuse the
group: rank 0 broadcasts each command and every node runs the same SPMD phase
sequence (services/service.py).  Control messages are length-prefixed JSON.
"""
from __future__ import annotations

import json
import os
import queue
import socket
import struct
import threading
import traceback

import torch

from ..crypto import oracle as O
from ..crypto.elgamal import CipherVector, KeyPair
from ..ledger.skipchain import SkipBlock
from ..parallel.topology import Cluster, Party
from ..utils.log import get_logger
from ..wire.messages import survey_query_from_wire, survey_query_to_wire

log = get_logger("server")


# ----------------------------------------------------------------------------- framing
def send_msg(sock: socket.socket, obj: dict):
    data = json.dumps(obj).encode()
    sock.sendall(struct.pack("<Q", len(data)) + data)


def recv_msg(sock: socket.socket) -> dict:
    hdr = _recv_exact(sock, 8)
    (n,) = struct.unpack("<Q", hdr)
    return json.loads(_recv_exact(sock, n).decode())


def _recv_exact(sock, n):
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(min(1 << 20, n - len(buf)))
        if not chunk:
            raise ConnectionError("peer closed")
        buf += chunk
    return bytes(buf)


def request(address: str, obj: dict, timeout: float = 3600.0) -> dict:
    host, port = address.rsplit(":", 1)
    with socket.create_connection((host, int(port)), timeout=timeout) as s:
        send_msg(s, obj)
        return recv_msg(s)


# ----------------------------------------------------------------------------- config
def gen_config(address: str, client_address: str = "", description: str = "") -> dict:
    """``server gen``: a new keypair + the node's config (TOML-able dict)."""
    kp = KeyPair.generate()
    return {"Address": address, "URL": client_address or address, "Description": description,
            "Public": O.g1_to_bytes(kp.public).hex(), "Private": O.scalar_to_bytes(kp.secret).hex(),
            "Suite": "bn256.G1"}


def node_id(address: str) -> str:
    return address


def cluster_from_roster(roles: dict, rank_of: dict, publics: dict, my_addr: str, my_key: KeyPair) -> Cluster:
    """roles: {"cn": [addr...], "dp": [...], "vn": [...]} -> logical parties on node ranks."""
    cl = Cluster(world=len(rank_of))
    for role, attr in (("cn", "cns"), ("dp", "dps"), ("vn", "vns")):
        for a in roles.get(role, []):
            p = Party(f"{role}:{a}", role, rank_of[a], O.g1_from_bytes(bytes.fromhex(publics[a])))
            if a == my_addr:
                p.keypair = my_key
            getattr(cl, attr).append(p)
    return cl


# ----------------------------------------------------------------------------- node server
class NodeServer:
    def __init__(self, config: dict, workdir: str | None = None, device=None):
        self.config = config
        self.address = config["Address"]
        self.key = KeyPair(int.from_bytes(bytes.fromhex(config["Private"]), "big"),
                           O.g1_from_bytes(bytes.fromhex(config["Public"])))
        self.workdir = workdir or os.path.join(os.getcwd(), "drynx_db_" + self.address.replace(":", "_"))
        self.device = device
        self.node = None          # DrynxNode once the group exists
        self.comm = None
        self.rank = None
        self.cmds: queue.Queue = queue.Queue()   # rank 0: (command, reply-queue)
        self._join_event = threading.Event()
        self._join_info = None
        self._stop = threading.Event()
        self._srv = None

    # --------------------------------------------------------------- TCP side
    def serve_forever(self):
        host, port = self.address.rsplit(":", 1)
        self._srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self._srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._srv.bind((host if host != "localhost" else "127.0.0.1", int(port)))
        self._srv.listen(64)
        threading.Thread(target=self._accept_loop, daemon=True).start()
        log.info(f"[SERVICE] <drynx> Server {self.address} listening")
        self._main_loop()

    def _accept_loop(self):
        while not self._stop.is_set():
            try:
                conn, _ = self._srv.accept()
            except OSError:
                return
            threading.Thread(target=self._handle_conn, args=(conn,), daemon=True).start()

    def _handle_conn(self, conn):
        try:
            msg = recv_msg(conn)
            cmd = msg.get("cmd")
            if cmd == "ping":
                send_msg(conn, {"ok": True, "address": self.address, "public": self.config["Public"]})
            elif cmd == "join":
                self._join_info = msg
                self._join_event.set()
                send_msg(conn, {"ok": True})
            else:
                if self.rank not in (None, 0):
                    send_msg(conn, {"ok": False, "error": "not the entry node of the running cluster"})
                    return
                reply: queue.Queue = queue.Queue()
                self.cmds.put((msg, reply))
                send_msg(conn, reply.get())
        except Exception as e:  # keep serving
            try:
                send_msg(conn, {"ok": False, "error": f"{type(e).__name__}: {e}"})
            except Exception:
                pass
        finally:
            conn.close()

    # --------------------------------------------------------------- cluster formation
    def _form_cluster_as_root(self, roster: list):
        """roster: list of node addresses (this node first)."""
        import torch.distributed as dist

        from ..parallel.comm import DistComm

        addrs = [self.address] + [a for a in roster if a != self.address]
        publics = {}
        for a in addrs:
            publics[a] = self.config["Public"] if a == self.address else request(a, {"cmd": "ping"})["public"]
        host = self.address.rsplit(":", 1)[0]
        host = "127.0.0.1" if host == "localhost" else host
        s = socket.socket()
        s.bind((host, 0))
        mport = s.getsockname()[1]
        s.close()
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        info = {"cmd": "join", "world": len(addrs), "master": f"{host}:{mport}", "backend": backend, "addrs": addrs,
                "publics": publics}
        for r, a in enumerate(addrs[1:], start=1):
            request(a, dict(info, rank=r))
        self._init_group(info, 0)
        return addrs, publics

    def _init_group(self, info, rank):
        import torch.distributed as dist

        from ..parallel.comm import DistComm

        host, port = info["master"].rsplit(":", 1)
        if info["backend"] == "nccl":
            torch.cuda.set_device(0)
        dist.init_process_group(info["backend"], init_method=f"tcp://{host}:{port}", rank=rank,
                                world_size=info["world"])
        self.comm = DistComm()
        self.rank = rank
        self.addrs = info["addrs"]
        self.publics = info["publics"]

    # --------------------------------------------------------------- main loop
    def _main_loop(self):
        # a node that is not contacted by a client waits for a join, then follows rank 0
        while not self._stop.is_set():
            if self.rank is None:
                got = None
                try:
                    got = self.cmds.get(timeout=0.2)
                except queue.Empty:
                    pass
                if got is not None:
                    msg, reply = got
                    if msg.get("cmd") == "survey":
                        self._form_cluster_as_root(msg["roster"])
                    self._dispatch_root(msg, reply)
                    continue
                if self._join_event.is_set():
                    self._init_group(self._join_info, self._join_info["rank"])
                continue
            if self.rank == 0:
                msg, reply = self.cmds.get()
                self._dispatch_root(msg, reply)
            else:
                cmd = self.comm.broadcast_object(None, src=0)
                if cmd is None or cmd.get("cmd") == "shutdown":
                    self._stop.set()
                    break
                self._execute(cmd)

    def _dispatch_root(self, msg, reply):
        try:
            if self.comm is not None:
                self.comm.broadcast_object(msg, src=0)
            out = self._execute(msg)
            reply.put(dict(out or {}, ok=True))
            if msg.get("cmd") == "shutdown":
                self._stop.set()
                if self._srv:
                    self._srv.close()
        except Exception as e:
            log.error(traceback.format_exc())
            reply.put({"ok": False, "error": f"{type(e).__name__}: {e}"})

    def _ensure_node(self, roles: dict):
        from .service import DrynxNode

        rank_of = {a: i for i, a in enumerate(self.addrs)}
        cl = cluster_from_roster(roles, rank_of, self.publics, self.address, self.key)
        if self.node is None or [p.id for p in self.node.cluster.parties] != [p.id for p in cl.parties]:
            self.node = DrynxNode(cl, self.comm, self.workdir, self.comm.device)
        return self.node

    def _execute(self, msg: dict):
        cmd = msg.get("cmd")
        if cmd == "survey":
            node = self._ensure_node(msg["roles"])
            # the survey travels as the reference's network.Marshal(&SurveyQuery)
            sq = survey_query_from_wire(bytes.fromhex(msg["sq"])) if self.rank == 0 else None
            res = node.run_survey(sq)
            if self.rank == 0:
                return {"survey_id": res.survey_id, "n_groups": res.n_groups, "n_out": res.n_out,
                        "cv": res.result.to_bytes().hex(),
                        "block": res.block.to_bytes().decode() if res.block is not None else None}
            return None
        if cmd in ("get_genesis", "get_latest_block", "get_block", "get_proofs", "close_db"):
            vn = msg["vn"]
            node = self.node
            owner = node.cluster.by_id(vn).rank if node else 0
            out = None
            if self.rank == owner and node is not None:
                if cmd == "get_genesis":
                    b = node.get_genesis(vn)
                    out = {"block": b.to_bytes().decode() if b else None}
                elif cmd == "get_latest_block":
                    b = node.get_latest_block(vn)
                    out = {"block": b.to_bytes().decode() if b else None}
                elif cmd == "get_block":
                    b = node.get_block(vn, msg["survey_id"])
                    out = {"block": b.to_bytes().decode() if b else None}
                elif cmd == "get_proofs":
                    out = {"proofs": {k: v.hex() for k, v in node.get_proofs(vn, msg["survey_id"]).items()}}
                else:
                    node.close_db(vn, bool(msg.get("remove")))
                    out = {}
            if self.comm is not None and self.comm.world > 1:
                outs = self.comm.all_gather_object(out)
                out = next((o for o in outs if o is not None), None)
            return out
        if cmd == "shutdown":
            return {}
        raise ValueError(f"unknown command {cmd}")


# ----------------------------------------------------------------------------- client-side proxy
class RemoteNode:
    """Entry point for ``DrynxClient`` talking to a running server over TCP."""

    def __init__(self, address: str, roles: dict, roster: list):
        self.address = address
        self.roles = roles
        self.roster = roster

    def run_survey(self, sq, on_result=None):
        from .service import SurveyResult

        out = request(self.address, {"cmd": "survey", "sq": survey_query_to_wire(sq).hex(), "roles": self.roles,
                                     "roster": self.roster})
        if not out.get("ok"):
            raise RuntimeError(out.get("error"))
        cv = CipherVector.from_bytes(bytes.fromhex(out["cv"]))
        blk = SkipBlock.from_bytes(out["block"].encode()) if out.get("block") else None
        res = SurveyResult(out["survey_id"], cv, out["n_groups"], out["n_out"], blk)
        if on_result is not None:
            res.client_out = on_result(res)
        return res

    def _vn(self, cmd, vn, **kw):
        out = request(self.address, dict({"cmd": cmd, "vn": vn}, **kw))
        if not out.get("ok"):
            raise RuntimeError(out.get("error"))
        return out

    def get_genesis(self, vn):
        b = self._vn("get_genesis", vn).get("block")
        return SkipBlock.from_bytes(b.encode()) if b else None

    def get_latest_block(self, vn):
        b = self._vn("get_latest_block", vn).get("block")
        return SkipBlock.from_bytes(b.encode()) if b else None

    def get_block(self, vn, survey_id):
        b = self._vn("get_block", vn, survey_id=survey_id).get("block")
        return SkipBlock.from_bytes(b.encode()) if b else None

    def get_proofs(self, vn, survey_id):
        return {k: bytes.fromhex(v) for k, v in self._vn("get_proofs", vn, survey_id=survey_id)["proofs"].items()}

    def close_db(self, vn, remove=False):
        self._vn("close_db", vn, remove=remove)

    def shutdown(self):
        try:
            request(self.address, {"cmd": "shutdown"}, timeout=30)
        except Exception:
            pass
