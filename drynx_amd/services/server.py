"""Standalone node servers + TCP control plane (the onet ``Server`` equivalent).

Reference: cmd/server/main.go (``gen`` keypair + config, ``run`` reads the
config and serves), the onet client API (services/api.go:39-133,
services/api_skipchain.go:16-106), and the multi-process test of test/lib.sh
(3 real servers on localhost).

Wire format: every control message is an onet envelope, ``network.Marshal`` =
16-byte message-type id + dedis/protobuf body (drynx_amd/wire/onet.py),
length-prefixed on a TCP stream.  The client speaks the reference's messages:
``libdrynx.SurveyQuery`` (reply ``libdrynx.ResponseDP``), ``SurveyQueryToVN``,
``EndVerificationRequest`` / ``GetGenesis`` / ``GetBlock`` /
``GetLatestBlock`` (reply ``libdrynx.Reply``), ``GetProofs`` (reply
``ProofsAsMap``) and ``CloseDB``; VN requests carry the VN id as an appended
field, since one entry node hosts many logical VNs.

Model: every ``server run`` process is one node (one GPU or one CPU worker)
with its own long-term key.  A client sends a survey to an entry node; its
roster (CNs, DPs, VNs with their public keys) comes from the SurveyQuery
itself.  On the first survey the entry node becomes rank 0 of a
torch.distributed group with the roster nodes (RCCL when every node has a
GPU, gloo otherwise):

* the entry node sends each node a ``drynx_amd.Join`` (world size, rank,
  rendezvous address, roster keys) Schnorr-signed with its node key over a
  fresh nonce;
* a node joins only if every roster key is in its group file (``Trusted``,
  from ``server run --group``), the signature verifies under the root's key,
  its own entry is its own address and key, and it is not already in a group;
  it answers with a signature of the nonce under its own key, which
  the root checks against the roster before the rendezvous.

Only authenticated roster members reach the process group, whose collectives
then carry the SPMD commands (services/service.py).  Residual exposure: the
rendezvous port of torch.distributed is open during the few seconds of group
formation.
"""
from __future__ import annotations

import hashlib
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
from ..proofs import sigma
from ..utils.log import get_logger
from ..wire import onet
from ..wire.messages import survey_query_from_msg, survey_query_to_msg

log = get_logger("server")


# ----------------------------------------------------------------------------- framing
def send_env(sock: socket.socket, env: bytes):
    sock.sendall(struct.pack("<Q", len(env)) + env)


# an unauthenticated peer's first frame (Ping, Join, SurveyQuery, VN calls) is a
# control message: capped well below anything that could exhaust host memory;
# only replies the caller asked for (proof maps, blocks) may be larger
CONTROL_FRAME_LIMIT = 64 << 20
REPLY_FRAME_LIMIT = 1 << 34


def recv_env(sock: socket.socket, limit: int = CONTROL_FRAME_LIMIT) -> bytes:
    (n,) = struct.unpack("<Q", _recv_exact(sock, 8))
    if n > limit:
        raise ValueError(f"frame of {n} bytes exceeds the limit of {limit}")
    return _recv_exact(sock, n)


def _recv_exact(sock, n):
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(min(1 << 20, n - len(buf)))
        if not chunk:
            raise ConnectionError("peer closed")
        buf += chunk
    return bytes(buf)


def request(address: str, go_type: str, fields: dict, timeout: float = 3600.0) -> tuple[str, dict]:
    """One onet message to ``address`` and its reply (name, fields).  A
    ``drynx_amd.Error`` reply raises."""
    host, port = address.rsplit(":", 1)
    with socket.create_connection((host, int(port)), timeout=timeout) as s:
        send_env(s, onet.marshal(go_type, fields))
        name, d = onet.unmarshal(recv_env(s, REPLY_FRAME_LIMIT))
    if name == "drynx_amd.Error":
        raise RuntimeError(d["Message"])
    return name, d


# ----------------------------------------------------------------------------- config
def gen_config(address: str, client_address: str = "", description: str = "") -> dict:
    """``server gen``: a new keypair + the node's config (TOML-able dict)."""
    kp = KeyPair.generate()
    return {"Address": address, "URL": client_address or address, "Description": description,
            "Public": O.g1_to_bytes(kp.public).hex(), "Private": O.scalar_to_bytes(kp.secret).hex(),
            "Suite": "bn256.G1"}


def roster_of_survey(sq) -> tuple[dict, dict]:
    """(roles {"cn"|"dp"|"vn": [address]}, {address: public}) from the query's
    CN roster, DP assignment and VN roster."""
    roles = {"cn": [], "dp": [], "vn": []}
    pubs: dict = {}

    def add(role, si):
        if si.address not in roles[role]:
            roles[role].append(si.address)
        if pubs.setdefault(si.address, si.public) != si.public:
            raise ValueError(f"two keys for node {si.address}")

    for si in sq.RosterServers.list:
        add("cn", si)
    for dps in (sq.ServerToDP or {}).values():
        for si in dps or []:
            add("dp", si)
    if sq.Query.RosterVNs is not None:
        for si in sq.Query.RosterVNs.list:
            add("vn", si)
    return roles, pubs


def cluster_from_roster(roles: dict, rank_of: dict, publics: dict, my_addr: str, my_key: KeyPair) -> Cluster:
    """roles: {"cn": [addr...], "dp": [...], "vn": [...]} -> logical parties on node ranks."""
    cl = Cluster(world=len(rank_of))
    for role, attr in (("cn", "cns"), ("dp", "dps"), ("vn", "vns")):
        for a in roles.get(role, []):
            p = Party(f"{role}:{a}", role, rank_of[a], publics[a])
            if a == my_addr:
                p.keypair = my_key
            getattr(cl, attr).append(p)
    return cl


def _join_digest(d: dict) -> bytes:
    body = onet.marshal("drynx_amd.Join", dict(d, Signature=b""))
    return hashlib.sha256(b"drynx_amd/join/v1" + body).digest()


def _abort_digest(nonce: bytes, address: str) -> bytes:
    return hashlib.sha256(b"drynx_amd/join-abort/v1" + nonce + address.encode()).digest()


JOIN_TIMEOUT_S = 120.0  # a joined node that never sees the rendezvous complete resets after this


def _ack_digest(nonce: bytes, address: str) -> bytes:
    return hashlib.sha256(b"drynx_amd/join-ack/v1" + nonce + address.encode()).digest()


def _reply_block(b: SkipBlock | None) -> tuple[str, dict]:
    return "libdrynx.Reply", {"Latest": b.to_bytes() if b is not None else b""}


# ----------------------------------------------------------------------------- node server
class NodeServer:
    def __init__(self, config: dict, workdir: str | None = None, device=None):
        self.config = config
        self.address = config["Address"]
        self.key = KeyPair(int.from_bytes(bytes.fromhex(config["Private"]), "big"),
                           O.g1_from_bytes(bytes.fromhex(config["Public"])))
        # the group file: keys of the nodes this node may form a cluster with
        # (``server run --group network.toml``); ``TrustAny`` accepts any root
        # (trust on first use, local experiments only)
        self.trusted = {bytes.fromhex(k) for k in config.get("Trusted", [])}
        self.trust_any = bool(config.get("TrustAny", False))
        self.workdir = workdir or os.path.join(os.getcwd(), "drynx_db_" + self.address.replace(":", "_"))
        # device of this node: --device, the config's Device, LOCAL_RANK, else GPU 0 / CPU
        dev = device or config.get("Device")
        if dev is None:
            dev = f"cuda:{int(os.environ.get('LOCAL_RANK', '0'))}" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(dev)
        self.node = None          # DrynxNode once the group exists
        self._node_ready = threading.Event()
        self.comm = None
        self.rank = None
        self.cmds: queue.Queue = queue.Queue()   # rank 0: (name, fields, reply-queue)
        self._join_lock = threading.Lock()
        self._join_info = None
        self._join_event = threading.Event()
        self._stop = threading.Event()
        self._srv = None
        self._pending_vn: dict = {}   # SurveyQueryToVN received before the group existed
        # roles this node serves (``server computing-node / verifying-node /
        # data-provider new``): None = any role (a config without role sections)
        offered = {r for r, sec in (("cn", "ComputingNode"), ("vn", "VerifyingNode"), ("dp", "DataProvider"))
                   if sec in config}
        self.offers = offered or None
        self.dp_source = config.get("DataProvider") or {}

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
                conn, peer = self._srv.accept()
            except OSError:
                return
            threading.Thread(target=self._handle_conn, args=(conn, peer), daemon=True).start()

    def _handle_conn(self, conn, peer):
        try:
            name, d = onet.unmarshal(recv_env(conn))
            out = self._handle_message(name, d, peer)
            send_env(conn, onet.marshal(*out))
        except Exception as e:  # keep serving
            try:
                send_env(conn, onet.marshal("drynx_amd.Error", {"Message": f"{type(e).__name__}: {e}"}))
            except Exception:
                pass
        finally:
            conn.close()

    def _handle_message(self, name: str, d: dict, peer) -> tuple[str, dict]:
        if name == "drynx_amd.Ping":
            return "drynx_amd.PingReply", {"Address": self.address, "Public": O.g1_to_bytes(self.key.public)}
        if name == "drynx_amd.Join":
            return self._accept_join(d)
        if name == "drynx_amd.JoinAbort":
            return self._abort_join(d)
        if name == "drynx_amd.Shutdown" and peer[0] not in ("127.0.0.1", "::1"):
            raise PermissionError("shutdown is accepted from the local host only")
        if name == "libdrynx.SurveyQueryToVN":
            sq = survey_query_from_msg(d["SQ"])
            if self.node is not None:
                self.node.register_vn_survey(sq)
            else:
                self._pending_vn[sq.SurveyID] = sq
            return "drynx_amd.Ack", {"OK": True}
        if name == "libdrynx.EndVerificationRequest":
            # blocks this connection only (the query itself may still be running)
            timeout = d["Timeout"] or 3600.0
            if not self._node_ready.wait(timeout):
                return _reply_block(None)
            return _reply_block(self.node.wait_end_verification(d["QueryInfoID"], timeout))
        if self.rank not in (None, 0):
            raise RuntimeError("not the entry node of the running cluster")
        reply: queue.Queue = queue.Queue()
        self.cmds.put((name, d, reply))
        out = reply.get()
        if isinstance(out, Exception):
            raise out
        return out

    # --------------------------------------------------------------- cluster formation
    def _accept_join(self, d: dict) -> tuple[str, dict]:
        with self._join_lock:
            if self.rank is not None or self._join_info is not None:
                raise PermissionError("already part of a cluster")
            addrs, pubs = list(d["Addrs"]), [bytes(p) for p in d["Publics"]]
            r = d["Rank"]
            if len(addrs) != d["World"] or len(pubs) != len(addrs) or not 0 < r < len(addrs):
                raise ValueError("malformed join")
            if addrs[r] != self.address or pubs[r] != O.g1_to_bytes(self.key.public):
                raise PermissionError("join does not name this node with its own key")
            if d["Root"] != addrs[0]:
                raise ValueError("the root must be rank 0")
            if not self.trusted and not self.trust_any:
                raise PermissionError("no group file: this node accepts no join")
            if self.trusted and not set(pubs) <= self.trusted:
                raise PermissionError("roster contains keys this node does not trust")
            root_pub = O.g1_from_bytes(pubs[0])
            if not sigma.schnorr_verify(root_pub, _join_digest(d), d["Signature"]):
                raise PermissionError("bad root signature on join")
            self._join_info = d
            self._join_time = __import__("time").monotonic()
        self._join_event.set()
        return "drynx_amd.JoinReply", {"Signature": sigma.schnorr_sign(self.key.secret,
                                                                       _ack_digest(d["Nonce"], self.address))}

    def _abort_join(self, d: dict) -> tuple[str, dict]:
        """The root gave up forming the cluster it invited this node to (signed
        by that root, bound to the join's nonce): forget the join."""
        with self._join_lock:
            info = self._join_info
            if info is None or self.rank is not None:
                return "drynx_amd.Ack", {"OK": False}
            if d["Root"] != info["Root"] or bytes(d["Nonce"]) != bytes(info["Nonce"]):
                raise PermissionError("abort does not match the pending join")
            root_pub = O.g1_from_bytes(bytes(info["Publics"][0]))
            if not sigma.schnorr_verify(root_pub, _abort_digest(bytes(d["Nonce"]), self.address), d["Signature"]):
                raise PermissionError("bad root signature on join abort")
            self._join_info = None
            self._join_event.clear()
        return "drynx_amd.Ack", {"OK": True}

    def _form_cluster_as_root(self, sq):
        roles, pubs = roster_of_survey(sq)
        addrs = [self.address]
        for role in ("cn", "dp", "vn"):
            addrs += [a for a in roles[role] if a not in addrs]
        if self.address in pubs and pubs[self.address] != self.key.public:
            raise PermissionError("the query names this node with another key")
        pubs[self.address] = self.key.public
        # the entry node applies its own group file to the client's roster
        # before contacting anyone: a client cannot make it form a (lasting)
        # process group with nodes it does not trust
        if not self.trusted and not self.trust_any:
            raise PermissionError("no group file: this node forms no cluster")
        if self.trusted and not {O.g1_to_bytes(pubs[a]) for a in addrs} <= self.trusted:
            raise PermissionError("the query's roster contains keys this node does not trust")
        host = self.address.rsplit(":", 1)[0]
        host = "127.0.0.1" if host == "localhost" else host
        s = socket.socket()
        s.bind((host, 0))
        mport = s.getsockname()[1]
        s.close()
        backend = "nccl" if self.device.type == "cuda" else "gloo"
        base = {"World": len(addrs), "Master": f"{host}:{mport}", "Backend": backend, "Addrs": addrs,
                "Publics": [O.g1_to_bytes(pubs[a]) for a in addrs], "Root": self.address}
        accepted = []
        try:
            for r, a in enumerate(addrs[1:], start=1):
                d = dict(base, Rank=r, Nonce=os.urandom(32))
                d["Signature"] = sigma.schnorr_sign(self.key.secret, _join_digest(d))
                name, rep = request(a, "drynx_amd.Join", d, timeout=60)
                accepted.append((a, d["Nonce"]))
                if name != "drynx_amd.JoinReply" or not sigma.schnorr_verify(pubs[a], _ack_digest(d["Nonce"], a),
                                                                              rep["Signature"]):
                    raise PermissionError(f"node {a} did not prove its roster key")
        except Exception:
            # the rendezvous will never complete: release the peers that accepted
            for a, nonce in accepted:
                abort = {"Root": self.address, "Nonce": nonce}
                abort["Signature"] = sigma.schnorr_sign(self.key.secret, _abort_digest(nonce, a))
                try:
                    request(a, "drynx_amd.JoinAbort", abort, timeout=10)
                except Exception:  # noqa: BLE001 -- best effort; the peer's join timeout covers the rest
                    pass
            raise
        self._init_group(dict(base, Rank=0), 0)

    def _init_group_or_reset(self, info):
        """Join the rendezvous; if it does not complete within JOIN_TIMEOUT_S
        (the root died or aborted), forget the join so a later one is accepted."""
        try:
            self._init_group(info, info["Rank"], timeout=JOIN_TIMEOUT_S)
        except Exception as e:  # noqa: BLE001 -- the rendezvous failed: back to waiting
            log.warning(f"cluster rendezvous failed ({type(e).__name__}: {e}); waiting for a new join")
            with self._join_lock:
                self._join_info = None
                self._join_event.clear()

    def _init_group(self, info, rank, timeout: float | None = None):
        import torch.distributed as dist

        from ..parallel.comm import DistComm

        host, port = info["Master"].rsplit(":", 1)
        if info["Backend"] == "nccl":
            torch.cuda.set_device(self.device)
        import datetime

        # the rendezvous (not the later collectives) is bounded: a member whose
        # root never completes it gives up after ``timeout``
        store = dist.TCPStore(host, int(port), info["World"], rank == 0,
                              timeout=datetime.timedelta(seconds=timeout or 1800))
        dist.init_process_group(info["Backend"], store=store, rank=rank, world_size=info["World"])
        self.comm = DistComm(self.device if info["Backend"] == "nccl" else "cpu")
        self.rank = rank
        self.addrs = list(info["Addrs"])
        self.publics = {a: O.g1_from_bytes(bytes(p)) for a, p in zip(info["Addrs"], info["Publics"])}

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
                    name, d, reply = got
                    if name == "libdrynx.SurveyQuery":
                        try:
                            self._form_cluster_as_root(survey_query_from_msg(d))
                        except Exception as e:
                            log.error(traceback.format_exc())
                            reply.put(e)
                            continue
                    self._dispatch_root(name, d, reply)
                    continue
                if self._join_event.is_set():
                    with self._join_lock:
                        info = self._join_info
                    if info is not None:
                        self._init_group_or_reset(info)
                continue
            if self.rank == 0:
                name, d, reply = self.cmds.get()
                self._dispatch_root(name, d, reply)
            else:
                cmd = self.comm.broadcast_object(None, src=0)
                if cmd is None or cmd[0] == "drynx_amd.Shutdown":
                    self._stop.set()
                    break
                self._execute(*cmd)

    def _dispatch_root(self, name, d, reply):
        try:
            if self.comm is not None:
                self.comm.broadcast_object((name, d), src=0)
            reply.put(self._execute(name, d))
            if name == "drynx_amd.Shutdown":
                self._stop.set()
                if self._srv:
                    self._srv.close()
        except Exception as e:
            log.error(traceback.format_exc())
            reply.put(e)

    def _check_roles(self, roles: dict):
        """Refuse a survey that gives a node a role its config does not offer:
        every rank checks its own config, one all-gather makes the refusal
        unanimous (no rank enters the survey's collectives alone)."""
        mine = {r for r, addrs in roles.items() if self.address in addrs}
        bad = sorted(mine - self.offers) if self.offers is not None else []
        msg = f"{self.address} does not serve {bad} (its server config offers {sorted(self.offers)})" if bad else ""
        msgs = self.comm.all_gather_object(msg) if self.comm is not None and self.comm.world > 1 else [msg]
        msgs = [m for m in msgs if m]
        if msgs:
            raise ValueError("; ".join(msgs))

    def _load_dp_data(self, node, sq, roles: dict):
        """A data provider configured with a file loader answers from its file
        (``server data-provider new file-loader PATH``) instead of the query's
        generated data: its party's records for this survey's operation."""
        if self.address not in roles.get("dp", []) or self.dp_source.get("Source") != "file-loader":
            return
        from ..models.datasets import load_dp_file

        node.dp_data[f"dp:{self.address}"] = load_dp_file(self.dp_source["Path"], sq.Query.Operation, node.device)

    def _ensure_node(self, roles: dict):
        from .service import DrynxNode

        rank_of = {a: i for i, a in enumerate(self.addrs)}
        cl = cluster_from_roster(roles, rank_of, self.publics, self.address, self.key)
        if self.node is None or [p.id for p in self.node.cluster.parties] != [p.id for p in cl.parties]:
            # VNs' BLS keys (skipchain collective signature): derived where the key lives, then shared
            from ..crypto import bls

            mine = {p.id: O.g2_to_bytes(bls.public_key(p.keypair.secret)) for p in cl.vns if p.keypair is not None}
            allb = {}
            for part in (self.comm.all_gather_object(mine) if self.comm.world > 1 else [mine]):
                allb.update(part)
            for p in cl.vns:
                p.bls_public = O.g2_from_bytes(allb[p.id])
            self.node = DrynxNode(cl, self.comm, self.workdir, self.comm.device)
            # every rank is a separate party here: each VN verifies on its own
            # rank, never through another party's pooled slice verdicts
            self.node.pool_policy = "0"
            for sq in self._pending_vn.values():
                self.node.register_vn_survey(sq)
            self._pending_vn.clear()
            self._node_ready.set()
        return self.node

    def _vn_call(self, name: str, d: dict):
        """A VN getter, answered by the rank hosting that VN."""
        vn = d["VN"]
        node = self.node
        owner = node.cluster.by_id(vn).rank if node else 0
        out = None
        if node is not None and self.rank == owner:
            if name == "libdrynx.GetGenesis":
                out = _reply_block(node.get_genesis(vn))
            elif name == "libdrynx.GetLatestBlock":
                sb = SkipBlock.from_bytes(d["Sb"]) if d["Sb"] else None
                out = _reply_block(node.get_latest_block(vn, sb))
            elif name == "libdrynx.GetBlock":
                out = _reply_block(node.get_block(vn, d["ID"]))
            elif name == "libdrynx.GetProofs":
                out = ("libdrynx.ProofsAsMap", {"Proofs": node.get_proofs(vn, d["ID"])})
            else:
                node.close_db(vn, bool(d["Close"]))
                out = ("drynx_amd.Ack", {"OK": True})
        if self.comm is not None and self.comm.world > 1:
            outs = self.comm.all_gather_object(out)
            out = next((o for o in outs if o is not None), None)
        if out is None:
            raise KeyError(f"unknown VN {vn}")
        return out

    def _execute(self, name: str, d: dict):
        if name == "libdrynx.SurveyQuery":
            sq = survey_query_from_msg(d)
            roles, _ = roster_of_survey(sq)
            self._check_roles(roles)
            node = self._ensure_node(roles)
            self._load_dp_data(node, sq, roles)
            res = node.run_survey(sq if self.rank == 0 else None)
            if self.rank != 0:
                return None
            n_out = res.n_out
            data = {}
            for g in range(res.n_groups):
                cv = res.result[g * n_out:(g + 1) * n_out]
                raw = cv.to_bytes()
                data[str(g)] = [{"K": raw[128 * i: 128 * i + 64], "C": raw[128 * i + 64: 128 * i + 128]}
                                for i in range(len(cv))]
            return "libdrynx.ResponseDP", {"Data": data, "SurveyID": res.survey_id,
                                           "Block": res.block.to_bytes() if res.block is not None else b""}
        if name in ("libdrynx.GetGenesis", "libdrynx.GetLatestBlock", "libdrynx.GetBlock", "libdrynx.GetProofs",
                    "libdrynx.CloseDB"):
            return self._vn_call(name, d)
        if name == "drynx_amd.Shutdown":
            return "drynx_amd.Ack", {"OK": True}
        raise ValueError(f"unsupported message {name}")


# ----------------------------------------------------------------------------- client-side proxy
class RemoteNode:
    """Entry point for ``DrynxClient`` talking to a running server over the
    onet-envelope TCP control plane."""

    def __init__(self, address: str):
        self.address = address

    def run_survey(self, sq, on_result=None):
        from .service import SurveyResult

        name, out = request(self.address, "libdrynx.SurveyQuery", survey_query_to_msg(sq))
        if name != "libdrynx.ResponseDP":
            raise RuntimeError(f"unexpected reply {name}")
        groups = sorted(out["Data"], key=int)
        parts = [b"".join(ct["K"] + ct["C"] for ct in out["Data"][g]) for g in groups]
        n_out = len(out["Data"][groups[0]]) if groups else 0
        cv = CipherVector.from_bytes(b"".join(parts))
        blk = SkipBlock.from_bytes(out["Block"]) if out["Block"] else None
        res = SurveyResult(out["SurveyID"], cv, len(groups), n_out, blk)
        if on_result is not None:
            res.client_out = on_result(res)
        return res

    def _block(self, go_type, fields, timeout=3600.0):
        _, d = request(self.address, go_type, fields, timeout)
        return SkipBlock.from_bytes(d["Latest"]) if d["Latest"] else None

    def register_vn_survey(self, sq):
        request(self.address, "libdrynx.SurveyQueryToVN", {"SQ": survey_query_to_msg(sq)})

    def wait_end_verification(self, survey_id, timeout=3600.0):
        return self._block("libdrynx.EndVerificationRequest", {"QueryInfoID": survey_id, "Timeout": timeout},
                           timeout + 30)

    def get_genesis(self, vn):
        return self._block("libdrynx.GetGenesis", {"VN": vn})

    def get_latest_block(self, vn, sb=None):
        return self._block("libdrynx.GetLatestBlock", {"VN": vn, "Sb": sb.to_bytes() if sb is not None else b""})

    def get_block(self, vn, survey_id):
        return self._block("libdrynx.GetBlock", {"VN": vn, "ID": survey_id})

    def get_proofs(self, vn, survey_id):
        _, d = request(self.address, "libdrynx.GetProofs", {"VN": vn, "ID": survey_id})
        return d["Proofs"]

    def close_db(self, vn, remove=False):
        request(self.address, "libdrynx.CloseDB", {"VN": vn, "Close": int(remove)})

    def shutdown(self):
        try:
            request(self.address, "drynx_amd.Shutdown", {}, timeout=30)
        except Exception:
            pass
