"""Roster -> GPU-rank placement of logical parties.

The reference runs every Computing Node (CN), Data Provider (DP) and
Verifying Node (VN) as its own onet server process (services/service_test.go
:29-66 slices one LocalTest roster into CN/DP/VN rosters; simul/drynx_simul.go
:308-333 does the same for the simulation).  Here a party is a logical entity
hosted by a rank (one rank per GPU); a rank hosts any number of parties and
all of them share its device buffers.  Placement is round-robin per role so
each role's work spreads over the xGMI-connected GPUs of the node.
"""
from __future__ import annotations

from dataclasses import dataclass, field

from ..crypto import bls
from ..crypto import oracle as O
from ..crypto.elgamal import KeyPair
from ..query import Roster, ServerIdentity


@dataclass
class Party:
    id: str
    role: str  # "cn" | "dp" | "vn"
    rank: int
    public: tuple = None
    keypair: KeyPair = None  # only set on the hosting rank
    bls_public: tuple = None  # VNs: G2 key of the skipchain collective signature

    def identity(self) -> ServerIdentity:
        return ServerIdentity(self.id, self.public, f"rank{self.rank}/{self.id}", self.rank, self.bls_public)


@dataclass
class Cluster:
    cns: list = field(default_factory=list)
    dps: list = field(default_factory=list)
    vns: list = field(default_factory=list)
    world: int = 1

    @property
    def parties(self):
        return self.cns + self.dps + self.vns

    def _ids(self) -> dict:
        """id -> (position, party), rebuilt when the party lists change size
        (thousands of DPs made the linear scan quadratic)."""
        n = (len(self.cns), len(self.dps), len(self.vns))
        idx = self.__dict__.get("_id_index")
        if idx is None or idx[0] != n:
            idx = (n, {p.id: (i, p) for i, p in enumerate(self.parties)})
            self.__dict__["_id_index"] = idx
        return idx[1]

    def by_id(self, pid: str) -> Party:
        e = self._ids().get(pid)
        if e is None:
            raise KeyError(pid)
        return e[1]

    def index_of(self, pid: str) -> int:
        e = self._ids().get(pid)
        if e is None:
            raise KeyError(pid)
        return e[0]

    def local(self, rank: int, role: str | None = None):
        return [p for p in self.parties if p.rank == rank and (role is None or p.role == role)]

    def roster_cns(self) -> Roster:
        return Roster([p.identity() for p in self.cns])

    def roster_vns(self) -> Roster:
        return Roster([p.identity() for p in self.vns])

    def server_to_dp(self) -> dict:
        """Assign each DP to a CN: prefer a CN on the DP's own rank (device-local
        hand-off, no xGMI hop), else round-robin (service_test.go repartitionDPs)."""
        out = {c.id: [] for c in self.cns}
        rr = 0
        for dp in self.dps:
            same = [c for c in self.cns if c.rank == dp.rank]
            if same:
                cn = same[len(out[same[0].id]) % len(same)] if len(same) > 1 else same[0]
            else:
                cn = self.cns[rr % len(self.cns)]
                rr += 1
            out[cn.id].append(dp.identity())
        return out


def build_cluster(n_cns: int, n_dps: int, n_vns: int, world: int = 1, rank: int = 0, comm=None,
                  deterministic_keys: bool = False, offsets: dict | None = None) -> Cluster:
    """Create parties, place them on ranks, generate each party's keys on its
    hosting rank and share only the public keys (all_gather_object).
    ``offsets[role]`` shifts a role's round robin (e.g. VNs after the CNs, so
    3 CNs and 3 VNs on an 8-GPU node occupy six different GPUs)."""
    off = {"cn": 0, "dp": 0, "vn": 0, **(offsets or {})}
    cl = Cluster(world=world)
    cl.cns = [Party(f"cn{i}", "cn", (off["cn"] + i) % world) for i in range(n_cns)]
    cl.dps = [Party(f"dp{i}", "dp", (off["dp"] + i) % world) for i in range(n_dps)]
    cl.vns = [Party(f"vn{i}", "vn", (off["vn"] + i) % world) for i in range(n_vns)]
    local_pub = {}
    for i, p in enumerate(cl.parties):
        if p.rank == rank:
            p.keypair = KeyPair.from_secret(1000 + i) if deterministic_keys else KeyPair.generate()
            p.public = p.keypair.public
            local_pub[p.id] = O.g1_to_bytes(p.public)
            if p.role == "vn":
                p.bls_public = bls.public_key(p.keypair.secret)
                local_pub[p.id + "#bls"] = O.g2_to_bytes(p.bls_public)
    if comm is not None and comm.world > 1:
        allpub = {}
        for d in comm.all_gather_object(local_pub):
            allpub.update(d)
    else:
        allpub = local_pub
    for p in cl.parties:
        if p.public is None:
            p.public = O.g1_from_bytes(allpub[p.id])
        if p.bls_public is None and p.id + "#bls" in allpub:
            p.bls_public = O.g2_from_bytes(allpub[p.id + "#bls"])
    return cl
