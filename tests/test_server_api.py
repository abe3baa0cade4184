"""Node-server control plane: authenticated cluster joins (group file, signed
join, signed acknowledgement) and the VN API over the onet-envelope TCP
protocol with real server processes (reference services/api_skipchain.go:
SendSurveyQueryToVNs, a blocking SendEndVerification, GetProofs, GetGenesis,
CloseDB)."""
import os
import socket
import subprocess
import sys
import threading
import time

import pytest

from drynx_amd.crypto import oracle as O
from drynx_amd.crypto.elgamal import KeyPair
from drynx_amd.proofs import sigma
from drynx_amd.services import server as srv

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cfg(addr, kp):
    return {"Address": addr, "Public": O.g1_to_bytes(kp.public).hex(), "Private": O.scalar_to_bytes(kp.secret).hex()}


def _join(root_kp, addrs, pubs, rank, signer=None):
    d = {"World": len(addrs), "Rank": rank, "Master": "127.0.0.1:1", "Backend": "gloo", "Addrs": addrs,
         "Publics": [O.g1_to_bytes(p) for p in pubs], "Root": addrs[0], "Nonce": os.urandom(32)}
    d["Signature"] = sigma.schnorr_sign((signer or root_kp).secret, srv._join_digest(d))
    return d


def test_join_requires_group_file_and_root_signature():
    a, b, evil = KeyPair.generate(), KeyPair.generate(), KeyPair.generate()
    addrs = ["127.0.0.1:7000", "127.0.0.1:7001"]
    trusted = [O.g1_to_bytes(k.public).hex() for k in (a, b)]
    # no group file: nobody may pull this node into a cluster
    n = srv.NodeServer(dict(_cfg(addrs[1], b)), device="cpu")
    with pytest.raises(PermissionError):
        n._accept_join(_join(a, addrs, [a.public, b.public], 1))
    n = srv.NodeServer(dict(_cfg(addrs[1], b), Trusted=trusted), device="cpu")
    # an untrusted root (its own key listed as the root's)
    with pytest.raises(PermissionError):
        n._accept_join(_join(evil, addrs, [evil.public, b.public], 1))
    # a trusted root's key but a signature by someone else
    with pytest.raises(PermissionError):
        n._accept_join(_join(a, addrs, [a.public, b.public], 1, signer=evil))
    # a join naming another key for this node
    with pytest.raises(PermissionError):
        n._accept_join(_join(a, addrs, [a.public, a.public], 1))
    assert n._join_info is None
    d = _join(a, addrs, [a.public, b.public], 1)
    name, rep = n._accept_join(d)
    assert name == "drynx_amd.JoinReply"
    assert sigma.schnorr_verify(b.public, srv._ack_digest(d["Nonce"], addrs[1]), rep["Signature"])
    with pytest.raises(PermissionError):  # one cluster per node
        n._accept_join(_join(a, addrs, [a.public, b.public], 1))


def test_join_abort_releases_the_node():
    a, b, evil = KeyPair.generate(), KeyPair.generate(), KeyPair.generate()
    addrs = ["127.0.0.1:7000", "127.0.0.1:7001"]
    n = srv.NodeServer(dict(_cfg(addrs[1], b), Trusted=[O.g1_to_bytes(k.public).hex() for k in (a, b)]),
                       device="cpu")
    d = _join(a, addrs, [a.public, b.public], 1)
    n._accept_join(d)
    forged = {"Root": addrs[0], "Nonce": d["Nonce"],
              "Signature": sigma.schnorr_sign(evil.secret, srv._abort_digest(d["Nonce"], addrs[1]))}
    with pytest.raises(PermissionError):  # only the inviting root can abort
        n._abort_join(forged)
    ok = {"Root": addrs[0], "Nonce": d["Nonce"],
          "Signature": sigma.schnorr_sign(a.secret, srv._abort_digest(d["Nonce"], addrs[1]))}
    assert n._abort_join(ok)[1]["OK"]
    assert n._join_info is None
    n._accept_join(_join(a, addrs, [a.public, b.public], 1))  # a new join is accepted again


def test_entry_node_checks_the_client_roster():
    """A client cannot make the entry node form a process group with nodes
    outside the entry node's own group file."""
    from drynx_amd.query import Operation, Query, Roster, ServerIdentity, SurveyQuery

    a, b, evil = KeyPair.generate(), KeyPair.generate(), KeyPair.generate()
    root = srv.NodeServer(dict(_cfg("127.0.0.1:7000", a), Trusted=[O.g1_to_bytes(k.public).hex() for k in (a, b)]),
                          device="cpu")
    si = lambda addr, kp: ServerIdentity(f"cn:{addr}", kp.public, addr)  # noqa: E731
    sq = SurveyQuery(SurveyID="s", RosterServers=Roster([si("127.0.0.1:7000", a), si("127.0.0.1:7666", evil)]),
                     ClientPubKey=b.public, ServerToDP={}, Query=Query(Operation=Operation()))
    with pytest.raises(PermissionError):
        root._form_cluster_as_root(sq)
    root2 = srv.NodeServer(dict(_cfg("127.0.0.1:7000", a)), device="cpu")  # no group file at all
    with pytest.raises(PermissionError):
        root2._form_cluster_as_root(sq)


def test_control_frames_are_bounded():
    import struct

    r, w = socket.socketpair()
    try:
        w.sendall(struct.pack("<Q", srv.CONTROL_FRAME_LIMIT + 1))
        with pytest.raises(ValueError):
            srv.recv_env(r)
    finally:
        r.close()
        w.close()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.slow
def test_vn_api_over_tcp(tmp_path):
    from drynx_amd.proofs import range_proof as rp
    from drynx_amd.query import QueryDPDataGen, Roster, ServerIdentity, choose_operation
    from drynx_amd.services.api import DrynxClient

    addrs = [f"127.0.0.1:{_port()}" for _ in range(2)]
    kps = [KeyPair.generate() for _ in addrs]
    group = "[Network]\n" + "".join(f'[[Network.Nodes]]\nAddress = "{a}"\n'
                                     f'PublicKey = "{O.g1_to_bytes(k.public).hex()}"\n'
                                     for a, k in zip(addrs, kps))
    (tmp_path / "group.toml").write_text(group)
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    procs = []
    try:
        for i, (a, k) in enumerate(zip(addrs, kps)):
            c = _cfg(a, k)
            toml = "[Server]\n" + "".join(f'{key} = "{v}"\n' for key, v in c.items())
            p = subprocess.Popen([sys.executable, "-m", "drynx_amd.cli.server", "run", "--workdir",
                                  str(tmp_path / f"n{i}"), "--device", "cpu", "--group", str(tmp_path / "group.toml")],
                                 stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                 cwd=ROOT, env=env)
            p.stdin.write(toml)
            p.stdin.close()
            procs.append(p)
        for a in addrs:
            for _ in range(300):
                try:
                    socket.create_connection(tuple([a.split(":")[0], int(a.split(":")[1])]), timeout=1).close()
                    break
                except OSError:
                    time.sleep(0.2)
        cn, dp, vn = (ServerIdentity(f"cn:{addrs[0]}", kps[0].public, addrs[0], 0),
                      ServerIdentity(f"dp:{addrs[1]}", kps[1].public, addrs[1], 1),
                      ServerIdentity(f"vn:{addrs[0]}", kps[0].public, addrs[0], 0))
        client = DrynxClient(srv.RemoteNode(addrs[0]))
        op = choose_operation("sum", 0, 40, 1, 0)
        sigs = [rp.init_range_proof_signatures([16])]
        sq = client.generate_survey_query(Roster([cn]), Roster([vn]), {cn.id: [dp]},
                                          {cn.id: cn.public, dp.id: dp.public, vn.id: vn.public}, "vn-api", op,
                                          [[16, 4]], sigs, 1, False, [1.0, 1.0, 1.0, 0.0, 1.0],
                                          dpdatagen=QueryDPDataGen([1], 10, 0, 40))
        client.send_survey_query_to_vns(sq)
        waited = {}
        t = threading.Thread(target=lambda: waited.setdefault("b", client.send_end_verification(vn.id, "vn-api")))
        t.start()  # blocks until the VNs are done (api_skipchain.go:30)
        _, vals, res = client.send_survey_query(sq)
        t.join(120)
        assert 0 <= vals[0][0] <= 400
        assert waited["b"] is not None and waited["b"].Hash == res.block.Hash
        assert set(res.block.data_block().Proofs.values()) == {1}
        assert client.send_get_genesis(vn.id).Hash == res.block.Hash
        assert client.send_get_latest_block(vn.id).Hash == res.block.Hash
        proofs = client.send_get_proofs(vn.id, "vn-api")
        assert any("/range/" in k for k in proofs) and all(isinstance(v, bytes) and v for v in proofs.values())
        client.send_close_db(vn.id)
    finally:
        srv.RemoteNode(addrs[0]).shutdown()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
