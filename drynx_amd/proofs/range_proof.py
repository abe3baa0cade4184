"""Pairing-based (Boneh–Boyen-signature, CCS08-style) range proofs, batched.

Reference: lib/range/range_proof.go
  * InitRangeProofSignature[Deterministic] (:249-288): CN key (x, y = xB) and
    u signatures A_k = (x+k)^-1 B2.
  * CreatePredicateRangeProofForAllServ (:320-407): prove that the ElGamal
    commitment C = mB + rP hides m = sum_j phi_j u^j with digits phi_j < u.
  * RangeProofVerification / RangeProofListVerification (:484-565).
  * ToBytes/FromBytes (:72-246) — field sizes kept (Challenge/Zr/Zphi/Zv 32 B,
    D 64 B, V 128 B, A 384 B, Commit 128 B).

MI355X design (all lists of proofs are processed as ONE batch on the device):
  prove : table-driven -- V = v A_phi from G2 comb / GLS tables of the
          signature points and a = e(B, A_phi)^{-s v} gT^t from GT tables
          (``SigMaterial.table_mode``: no pairing per item); without tables
          (too many distinct points for HBM) a_ij = FE(ML(-s_j B, V_ij)) *
          gT^{t_j} (fused kernel dx_rp_prove_a).  D = (sum u^j s_j) B +
          (sum m_j) P by two fixed-base mults; all Fr arithmetic on device.
  verify: the l*S pairing equations of every proof of the batch combined
          with each verifier's random GLV weights rho and regrouped by
          bilinearity (``verify_range_proof_list_multi``, dx_rpmsm.hip):
          e(B, R) prod_(p,i) e(-c_p y_pi, U_pi) with R one G2 MSM and U_pi
          the l-digit combinations -- n*S + 1 Miller loops per verifier and
          one final exponentiation; the prod a^rho side is a GT bucket
          multi-exponentiation, the D-equations one MSM.  The reference's
          AND over the list (:497-500) makes this exact up to a 2^-64
          soundness error; a failing batch is attributed per request.

Extension (documented): ranges may carry a third element ``offset``; the
proof then shows m + offset in [0, u^l) (signed values such as logistic-
regression coefficients).  offset = 0 is the reference behaviour.
"""
from __future__ import annotations

import hashlib
import io
import math
import os
import threading
from dataclasses import dataclass

import numpy as np
import torch

from .. import native as nt
from ..crypto import bn254 as bn
from ..crypto import oracle as O
from ..crypto.elgamal import CipherVector, pk_table
from ..query import PublishSignatureBytes
from ..utils import streams, timers
from ..utils.log import get_logger

log = get_logger("range_proof")

G2_LEN, G1_LEN, GT_LEN, SC_LEN = 128, 64, 384, 32


def _gamma_bits() -> int:
    """Bits of the per-VN GT-membership combination weights: 40 (the
    cyclotomic cofactor's smallest prime factor is ~2^38.8, so fewer bits
    would let a non-GT element pass with non-negligible probability).
    DRYNX_GAMMA_BITS may only raise it (up to 64)."""
    gb = int(os.environ.get("DRYNX_GAMMA_BITS", "40"))
    if not 40 <= gb <= 64:
        raise ValueError(f"DRYNX_GAMMA_BITS={gb}: the GT-membership weights need 40..64 bits")
    return gb


# ----------------------------------------------------------------------------- setup (CN side)

def init_range_proof_signature(u: int, secret: int | None = None, device="cpu") -> PublishSignatureBytes:
    """A CN's input-validation key for one output column: y = x*B, A_k = (x+k)^-1 * B2."""
    x = O.random_scalar() if secret is None else secret % O.R
    y = bn.g1_mul_point(x)
    inv = [pow((x + k) % O.R, -1, O.R) for k in range(u)]
    A = nt.g2_fb_mul(bn.base2_table(device), bn.scalars_tensor(inv, device))
    return PublishSignatureBytes(O.g1_to_bytes(y), bn.g2_aff_to_bytes(A).tobytes())


def init_range_proof_signatures(us: list, device="cpu") -> list:
    """Batched InitRangeProofSignature for many (CN, column) keys at once
    (range_proof.go:270-288, simul/drynx_simul.go:292-296): one random secret
    x per entry of ``us`` (ChaCha20 keyed from the OS CSPRNG, expanded on the
    device), y = x*B and every A_k = (x+k)^-1 * B2 -- the Fr additions and
    inversions row-wise on the device too -- in two fixed-base launches, so
    the 3 x 1M keys of a million-value range cost seconds, not minutes of
    Python big-int inversions.  The secrets never leave the device."""
    n = len(us)
    if n == 0:
        return []
    dev = torch.device(device)
    xs = nt.prg_scalars(os.urandom(32), n, dev)  # [n, 8] uniform nonzero Fr
    y = nt.g1_to_affine(nt.g1_fb_mul(bn.base_table(dev), xs))
    y_bytes = bn.g1_aff_to_bytes(y)
    u_t = torch.as_tensor([int(u) for u in us], dtype=torch.long)
    umax = int(u_t.max())
    ks = bn.scalars_tensor(range(umax), dev)  # [umax, 8]: k = 0 .. umax - 1
    # row (x_i + k) for every (i, k < u_i), in (i, k) order
    rows = torch.arange(umax).expand(n, umax) < u_t[:, None]
    xi = torch.arange(n)[:, None].expand(n, umax)[rows].to(dev)
    kk = torch.arange(umax)[None, :].expand(n, umax)[rows].to(dev)
    inv = nt.fr_arith(nt.FR_INV, nt.fr_arith(nt.FR_ADD, xs.index_select(0, xi).contiguous(),
                                             ks.index_select(0, kk).contiguous()))
    A = bn.g2_aff_to_bytes(nt.g2_fb_mul(bn.base2_table(dev), inv))
    out, o = [], 0
    for i, u in enumerate(us):
        out.append(PublishSignatureBytes(y_bytes[i].tobytes(), A[o: o + int(u)].tobytes()))
        o += int(u)
    return out


def init_range_proof_signature_deterministic(u: int, device="cpu") -> PublishSignatureBytes:
    """InitRangeProofSignatureDeterministic: x = 12 (range_proof.go:249)."""
    return init_range_proof_signature(u, 12, device)


class SigMaterial:
    """Device-resident view of InputValidationSigs[cn][col]: y_{i,col} (G1) and
    A_{i,col,k} (G2 affine), plus per-column Y = sum_i y_{i,col} bytes for the
    Fiat–Shamir hash."""

    def __init__(self, sigs, device="cpu"):
        """Vectorised over every (CN, column) key: one bytes join, one device
        decode (on-curve checked) of all y, the per-column sums of the y on
        the device, and numpy deduplication of keys and signature points (a
        million-value range brings 3 x 1M keys and 6M signature points)."""
        self.device = torch.device(device)
        self.S = len(sigs)
        self.n_cols = len(sigs[0]) if self.S else 0
        self.u = [len(sigs[0][c].Signature) // G2_LEN for c in range(self.n_cols)]
        self.umax = max(self.u) if self.u else 0
        flat_sigs = [s for row in sigs for s in row]  # index i*n_cols + c
        N = len(flat_sigs)
        pub = np.frombuffer(b"".join(bytes(s.Public) for s in flat_sigs), dtype=np.uint8)
        if pub.size != 64 * N:
            raise ValueError("input-validation keys must be 64-byte G1 points")
        pub = pub.reshape(N, 64)
        self._pub = pub
        y_aff = bn.g1_aff_from_bytes(pub, device, check=True) if N else None  # [N, 16]
        self.y_jac = nt.g1_from_affine(y_aff) if N else None
        umax = max(1, self.umax)
        lens = {len(s.Signature) for s in flat_sigs}
        if lens == {umax * G2_LEN}:  # every column the same u: one join
            A_bytes = np.frombuffer(b"".join(bytes(s.Signature) for s in flat_sigs), dtype=np.uint8).reshape(
                self.S, self.n_cols, umax, G2_LEN)
        else:
            A_bytes = np.zeros((self.S, self.n_cols, umax, G2_LEN), dtype=np.uint8)
            for q, s in enumerate(flat_sigs):
                raw = np.frombuffer(s.Signature, dtype=np.uint8).reshape(-1, G2_LEN)
                A_bytes[q // max(1, self.n_cols), q % max(1, self.n_cols), : raw.shape[0]] = raw
        flat = A_bytes.reshape(-1, G2_LEN)
        nz = flat.any(axis=1)
        A = torch.zeros((flat.shape[0], 32), dtype=torch.int32, device=device)
        if nz.any():
            if nz.all():
                A = bn.g2_aff_from_bytes(flat, device, check=False)
            else:
                A[torch.from_numpy(np.nonzero(nz)[0]).to(device)] = bn.g2_aff_from_bytes(flat[nz], device, check=False)
        self.A = A  # index (i*n_cols + c)*umax + k
        # per-column sum_i y_{i,col} (the Fiat-Shamir hash input), on the device
        if N:
            yj = self.y_jac.view(self.S, self.n_cols, -1)
            acc = yj[0].contiguous()
            for i in range(1, self.S):
                acc = nt.g1_add(acc, yj[i].contiguous())
            self._ysum = bn.g1_aff_to_bytes(nt.g1_to_affine(acc))  # [n_cols, 64]
        else:
            self._ysum = np.zeros((0, 64), dtype=np.uint8)
        # prover tables, keyed by the distinct signature point (deduplicated by value)
        _, first, inv = np.unique(np.ascontiguousarray(flat).view(np.dtype((np.void, G2_LEN))).reshape(-1),
                                  return_index=True, return_inverse=True)
        self.canon = torch.from_numpy(first[inv.reshape(-1)].astype(np.int64))  # A index -> first equal index
        self._ptab = {}
        # distinct CN keys y_{i,col} (one per CN when the signature sets reuse
        # a key, as InitRangeProofSignatureDeterministic does): comb tables let
        # the verifier's c*y_i be fixed-base multiplications
        if N:
            _, yfirst, yinv = np.unique(pub.view(np.dtype((np.void, 64))).reshape(-1), return_index=True,
                                        return_inverse=True)
            order = np.argsort(yfirst, kind="stable")  # slots in order of first appearance
            rank = np.empty_like(order)
            rank[order] = np.arange(order.size)
            self.y_slot = rank[yinv.reshape(-1)].tolist()
            self._y_first = yfirst[order]
            self._y_aff = y_aff
        else:
            self.y_slot, self._y_first, self._y_aff = [], np.zeros(0, dtype=np.int64), None
        self._ytab = {}

    @property
    def Ysum_bytes(self) -> list:
        """Per column: the encoding of sum_i y_{i,col} (range_proof.go:350-374)."""
        if not hasattr(self, "_ysum_list"):
            self._ysum_list = [r.tobytes() for r in self._ysum]
        return self._ysum_list

    @property
    def y_pts(self):
        """Oracle points of the keys, index i*n_cols + c (decoded on demand)."""
        pub = self._pub

        class _Lazy:
            def __getitem__(self, q):
                return O.g1_from_bytes(pub[q].tobytes())

            def __len__(self):
                return pub.shape[0]
        return _Lazy()

    @property
    def y_distinct(self) -> list:
        return [O.g1_from_bytes(self._pub[q].tobytes()) for q in self._y_first]

    def challenge_words(self, device):
        """(B encoding [16], per-column sum_i y_i encodings [n_cols, 16]) as
        little-endian int32 words for the device challenge hash."""
        key = ("cw", str(torch.device(device)))
        if key not in self._ytab:
            b = np.frombuffer(O.g1_to_bytes(O.G1_GEN), dtype="<i4").copy()
            y = np.ascontiguousarray(self._ysum).view("<i4").reshape(-1, 16).copy()
            self._ytab[key] = bn.publish(torch.from_numpy(b).to(device), torch.from_numpy(y).to(device))
        return self._ytab[key]

    def y_tables(self, device):
        """(comb tables [n_distinct*8192, 16], slot per y index) or None when
        the distinct keys' tables exceed the budget (0.5 MiB each: on a GPU up
        to ``DRYNX_Y_TABLES_MB``, default 16 GiB of HBM -- the reference's
        random per-CN, per-column keys of a SPECTF query are 6210 keys, 3 GiB
        -- so the verifier's c * y_i are fixed-base; 256 keys on the host)."""
        dev = torch.device(device)
        cap = (int(os.environ.get("DRYNX_Y_TABLES_MB", 16384)) << 20) // (8192 * 64) if dev.type == "cuda" else 256
        nd = len(self._y_first)
        if not nd or nd > cap:
            return None
        key = str(torch.device(device))
        if key not in self._ytab:
            aff = self._y_aff.index_select(0, torch.from_numpy(self._y_first.astype(np.int64)).to(
                self._y_aff.device)).to(device).contiguous()
            self._ytab[key] = bn.publish(nt.g1_fb_table(aff), torch.tensor(self.y_slot, dtype=torch.int32,
                                                                             device=device))
        return self._ytab[key]

    def attach_shard(self, comm, every_rank_proves: bool):
        """Build the GLS / 4-bit prover tables sharded over ``comm``'s ranks:
        rank k computes points [k n / W, (k+1) n / W) and every slice is then
        broadcast over the data plane (RCCL over xGMI) into each rank's full
        table, instead of every rank computing all of it.  Collective: only
        when EVERY rank proves (each calls the table build in the same query
        at the same point of its schedule); the layout choice is agreed on
        first (``table_mode``)."""
        if comm is not None and getattr(comm, "world", 1) > 1 and every_rank_proves:
            self._shard = comm
        else:
            self._shard = None

    def table_mode(self, device) -> int:
        """Prover comb-table layout for this signature set on ``device``:
        8 (8-bit combs, 4 MiB per distinct point: few distinct points, e.g.
        InitRangeProofSignatureDeterministic), 7 (GLS-2 tables with signed
        8-bit windows, 1.09 MiB per point, 34 additions per evaluation: the
        reference's random per-CN, per-column keys -- 99,360 points for a
        SPECTF-shaped query with 3 CNs and u = 16, ~111 GB of HBM), 6 (GLS-2
        with unsigned 6-bit windows, 693 KiB per point, 44 additions), 4 (4-bit
        combs, 480 KiB per point, 64 additions) or 0 (no
        tables: variable-base G2 + one pairing per item).  Budgets:
        ``DRYNX_PROVER_TABLE_MB`` (8-bit, default 8 GiB on a GPU / 96 MiB on the
        host) and ``DRYNX_PROVER_TABLE4_MB`` (GLS / 4-bit layouts, default: the
        free HBM minus the verifier's reserve ``DRYNX_VERIFY_RESERVE_GB`` = 48,
        at most 85% of it / 64 MiB on the host): a 3-CN SPECTF-shaped set
        (99,360 points) takes the GLS-8 layout (~111 GB), a 6-CN one (198,720
        points) the GLS-6 one (~138 GB)."""
        dev = torch.device(device)
        key = ("mode", str(dev))
        if key in self._ptab:
            return self._ptab[key]
        n = self.n_distinct
        forced = os.environ.get("DRYNX_PROVER_TABLE_BITS")
        b8 = int(os.environ.get("DRYNX_PROVER_TABLE_MB", 8192 if dev.type == "cuda" else 96)) << 20
        if "DRYNX_PROVER_TABLE4_MB" in os.environ:
            b4 = int(os.environ["DRYNX_PROVER_TABLE4_MB"]) << 20
        elif dev.type == "cuda":
            # the tables live as long as the signature set: what the rank keeps
            # free for everything else -- the verifier's per-query working set
            # (line / U images, bucket plans, joint tables: ~25 GB for a 1e6-item
            # inbox) and the ledger's staging -- is reserved first
            free = torch.cuda.mem_get_info(dev)[0]
            reserve = int(float(os.environ.get("DRYNX_VERIFY_RESERVE_GB", "48")) * (1 << 30))
            b4 = max(0, min(int(0.85 * free), free - reserve))
        else:
            b4 = 64 << 20
        if forced in ("0", "4", "6", "7", "8"):
            mode = int(forced)
        elif n * (4 << 20) <= b8:
            mode = 8
        elif n * nt.GLS8_ENTRIES * (128 + 384) <= b4:
            mode = 7
        elif n * nt.GLS6_ENTRIES * (128 + 384) <= b4:
            mode = 6
        elif n * nt.FB4_ENTRIES * (128 + 384) <= b4:
            mode = 4
        else:
            mode = 0
        shard = getattr(self, "_shard", None)
        if shard is not None and forced is None:
            # sharded builds need ONE layout on every rank: the most compact one any rank chose
            order = [8, 7, 6, 4, 0]
            mode = max(shard.all_gather_object(mode), key=order.index)
        self._ptab[key] = mode
        return mode

    def _host_tables_pay(self, n_points: int, n_items: int | None) -> bool:
        """Host cost model: a comb table costs thousands of G2 / GT additions
        per distinct point (an 8-bit comb: 8192 entries), while proving one
        item without it costs one variable-base G2 multiplication and one
        pairing -- ~64 items per distinct point before the table breaks even.
        Tables are built once the set's cumulative items per distinct point
        reach that (``DRYNX_HOST_TABLE_MIN_USES``): a one-shot CPU query (the
        simulation, BASELINE config 1) proves without them; a set reused
        query after query gets them.  A forced ``DRYNX_PROVER_TABLE_BITS``
        bypasses the model."""
        if os.environ.get("DRYNX_PROVER_TABLE_BITS") is not None or getattr(self, "_host_ok", False):
            return True  # forced, or the tables are (being) built: using them is free
        need = int(os.environ.get("DRYNX_HOST_TABLE_MIN_USES", "64"))
        if getattr(self, "_shard", None) is not None:
            # a sharded build is collective, so every rank must decide the same
            # without a control round: count the set's proving batches (every
            # rank proves once per query) instead of this rank's own items
            self._host_calls = getattr(self, "_host_calls", 0) + 1
            ok = self._host_calls >= need
        else:
            self._host_items = getattr(self, "_host_items", 0) + int(n_items if n_items is not None else n_points)
            ok = self._host_items >= need * max(1, self.n_distinct)
        self._host_ok = ok
        return ok

    def table_bytes(self) -> int:
        """HBM held by this set's prover and verifier (c * y_i) tables."""
        tot = 0
        for v in list(self._ptab.values()) + list(self._ytab.values()):
            if isinstance(v, tuple):
                tot += sum(t.numel() * t.element_size() for t in v if isinstance(t, torch.Tensor))
            elif isinstance(v, dict):
                tot += sum(t.numel() * t.element_size() for t in (v.get("g2"), v.get("gt")) if t is not None)
        return tot

    @property
    def n_distinct(self) -> int:
        if not hasattr(self, "_n_distinct"):
            self._n_distinct = int(torch.unique(self.canon).numel())
        return self._n_distinct

    def _prover_tables4(self, dev, mode: int = 4):
        """4-bit comb, GLS-2 6-bit (``mode`` 6) or GLS-2 signed 8-bit (7) tables
        of EVERY distinct signature point of the set, built once (chunked) and
        kept in HBM for the set's lifetime; -> (g2, gt, slot of each A index)."""
        key = (mode, str(dev))
        if key not in self._ptab:
            uniq, slot = torch.unique(self.canon, return_inverse=True)
            n = uniq.numel()
            E, g2_tab, gt_tab = {4: (nt.FB4_ENTRIES, nt.g2_fb4_table, nt.gt_fb4_table),
                                 6: (nt.GLS6_ENTRIES, nt.g2_gls6_table, nt.gt_gls6_table),
                                 7: (nt.GLS8_ENTRIES, nt.g2_gls8_table, nt.gt_gls8_table)}[mode]
            g2 = torch.empty((n * E, 32), dtype=torch.int32, device=dev)
            gt = torch.empty((n * E, 96), dtype=torch.int32, device=dev)
            A = self.A.to(dev)
            step = 8192
            shard = getattr(self, "_shard", None)
            W, k = (shard.world, shard.rank) if shard is not None else (1, 0)
            per = -(-n // W)
            bounds = [(min(n, r * per), min(n, (r + 1) * per)) for r in range(W)]
            lo, hi = bounds[k]
            with timers.span("rp.prove.tables4"):
                for a in range(lo, hi, step):
                    b = min(hi, a + step)
                    pts = A.index_select(0, uniq[a:b].to(dev)).contiguous()
                    g2_tab(pts, out=g2[a * E: b * E])
                    gphi = nt.pairing(bn.g1_generator_aff(dev).expand(b - a, 16).contiguous(), pts)
                    gt_tab(gphi, out=gt[a * E: b * E])
            if shard is not None:
                with timers.span("rp.prove.tables4.share"):
                    for r, (a, b) in enumerate(bounds):
                        if b > a:
                            shard.broadcast_into(g2[a * E: b * E], r)
                            shard.broadcast_into(gt[a * E: b * E], r)
            self._ptab[key] = bn.publish(g2, gt, slot.to(dev))
        return self._ptab[key]

    def prover_tables(self, a_idx: torch.Tensor, device, n_items: int | None = None):
        """Comb tables (G2 for V = v*A, GT for e(B, A)) of the distinct signature
        points used by a proof batch, cached for the lifetime of the signature
        set.  Returns (g2_tables, gt_tables, slot[a_idx-position], wbits) or
        None when no table layout fits the memory budget (``table_mode``) or,
        on the host, while the set has not yet been used enough to repay the
        build (``_host_tables_pay``)."""
        dev = torch.device(device)
        if dev.type == "cpu" and not self._host_tables_pay(a_idx.numel(), n_items):
            return None
        mode = self.table_mode(dev)
        if mode == 0:
            return None
        if mode in (4, 6, 7):
            g2, gt, slot = self._prover_tables4(dev, mode)
            return g2, gt, slot.index_select(0, a_idx.to(dev)), mode
        canon = self.canon.to(a_idx.device).index_select(0, a_idx)
        uniq, inv = torch.unique(canon, return_inverse=True)
        key = str(dev)
        cache = self._ptab.setdefault(key, {"idx": [], "g2": None, "gt": None, "pos": {}})
        missing = [int(u) for u in uniq.tolist() if int(u) not in cache["pos"]]
        if missing:
            pts = self.A.to(dev).index_select(0, torch.tensor(missing, dtype=torch.long, device=dev)).contiguous()
            g2 = nt.g2_fb_table(pts)
            gphi = nt.pairing(bn.g1_generator_aff(dev).expand(len(missing), 16).contiguous(), pts)
            gt = nt.gt_fb_table(gphi)
            cache["g2"] = g2 if cache["g2"] is None else torch.cat([cache["g2"], g2])
            cache["gt"] = gt if cache["gt"] is None else torch.cat([cache["gt"], gt])
            bn.publish(cache["g2"], cache["gt"])
            for m in missing:
                cache["pos"][m] = len(cache["idx"])
                cache["idx"].append(m)
        slot_of_uniq = torch.tensor([cache["pos"][int(u)] for u in uniq.tolist()], dtype=torch.long, device=dev)
        return cache["g2"], cache["gt"], slot_of_uniq.index_select(0, inv.to(dev)), 8


_gt_cache: dict = {}


def gt_generator_table(device="cpu"):
    """gT = e(B, B2) and its comb table (3 MiB of HBM, cached per device)."""
    key = str(torch.device(device))
    if key not in _gt_cache:
        gT = nt.pairing(bn.g1_generator_aff(device), bn.g2_generator_aff(device))
        _gt_cache[key] = bn.publish(gT, nt.gt_fb_table(gT))
    return _gt_cache[key]


# ----------------------------------------------------------------------------- proof list (columnar)
@dataclass
class RangeProofList:
    """n proofs sharing (u, l, S).  Tensors on one device."""
    u: int
    l: int
    S: int
    offset: list
    cols: list
    commit: CipherVector          # n ciphertexts (Commit)
    challenge: torch.Tensor = None  # [n, 8]
    zr: torch.Tensor = None         # [n, 8]
    D: torch.Tensor = None          # [n, 24] Jacobian
    zphi: torch.Tensor = None       # [n*l, 8]
    zv: torch.Tensor = None         # [n*S*l, 8]  index (p*S+i)*l+j
    V: torch.Tensor = None          # [n*S*l, 32]
    A: torch.Tensor = None          # [n*S*l, 96]

    def __len__(self):
        return len(self.commit)

    @property
    def has_rp(self) -> bool:
        return not (self.u == 0 and self.l == 0)

    # ------------------------------------------------------------- wire
    def to_bytes(self) -> bytes:
        """Columnar kyber-layout encoding of the list (all proofs share u,l,S)."""
        n = len(self)
        out = io.BytesIO()
        hdr = np.array([n, self.u, self.l, self.S], dtype="<i8")
        out.write(hdr.tobytes())
        out.write(np.asarray(self.offset, dtype="<i8").tobytes())
        out.write(np.asarray(self.cols, dtype="<i8").tobytes())
        out.write(self.commit.to_bytes())
        if self.has_rp and n:
            out.write(bn.scalars_to_bytes(self.challenge).tobytes())
            out.write(bn.scalars_to_bytes(self.zr).tobytes())
            out.write(bn.g1_aff_to_bytes(nt.g1_to_affine(self.D)).tobytes())
            out.write(bn.scalars_to_bytes(self.zv).tobytes())
            out.write(bn.scalars_to_bytes(self.zphi).tobytes())
            out.write(bn.g2_aff_to_bytes(self.V).tobytes())
            out.write(bn.gt_to_bytes(self.A).tobytes())
        return out.getvalue()

    @staticmethod
    def from_bytes(b: bytes, device="cpu") -> "RangeProofList":
        mv = memoryview(b)
        n, u, l, S = (int(v) for v in np.frombuffer(mv[:32], dtype="<i8"))
        off = 32
        offset = np.frombuffer(mv[off: off + 8 * n], dtype="<i8").tolist()
        off += 8 * n
        cols = np.frombuffer(mv[off: off + 8 * n], dtype="<i8").tolist()
        off += 8 * n
        commit = CipherVector.from_bytes(bytes(mv[off: off + 128 * n]), device)
        off += 128 * n
        rpl = RangeProofList(u, l, S, offset, cols, commit)
        if rpl.has_rp and n:
            def take(nbytes):
                nonlocal off
                chunk = bytes(mv[off: off + nbytes])
                off += nbytes
                return np.frombuffer(chunk, dtype=np.uint8)
            rpl.challenge = bn.scalars_from_bytes(take(SC_LEN * n), device)
            rpl.zr = bn.scalars_from_bytes(take(SC_LEN * n), device)
            rpl.D = nt.g1_from_affine(bn.g1_aff_from_bytes(take(G1_LEN * n), device))
            rpl.zv = bn.scalars_from_bytes(take(SC_LEN * n * S * l), device)
            rpl.zphi = bn.scalars_from_bytes(take(SC_LEN * n * l), device)
            rpl.V = bn.g2_aff_from_bytes(take(G2_LEN * n * S * l), device)
            rpl.A = bn.gt_from_bytes(take(GT_LEN * n * S * l), device)
        return rpl

    # ------------------------------------------------------------- raw (HBM-native) format
    def pack(self) -> torch.Tensor:
        """One int32 device tensor with every field as raw Montgomery limbs —
        the intra-cluster format (RCCL payload, VN store); ``to_bytes`` is the
        kyber-layout export."""
        dev = self.commit.device
        n, l, S = len(self), self.l, self.S
        meta = torch.tensor([0x52505231, n, self.u, l, S], dtype=torch.int32)
        offs = (torch.tensor(self.offset, dtype=torch.int64).view(torch.int32) if n
                else torch.empty(0, dtype=torch.int32))
        cols = torch.tensor(self.cols, dtype=torch.int32)
        parts = [meta.to(dev), offs.to(dev), cols.to(dev), self.commit.K.reshape(-1), self.commit.C.reshape(-1)]
        if self.has_rp and n:
            parts += [t.reshape(-1) for t in (self.challenge, self.zr, self.D, self.zphi, self.zv, self.V, self.A)]
        return torch.cat(parts)

    @staticmethod
    def unpack(t: torch.Tensor, meta=None, offs=None, cols=None) -> "RangeProofList":
        """Views into a packed list; ``meta``/``offs``/``cols`` may be given when
        the caller already fetched the header words (batched unpack)."""
        if meta is None:
            meta = t[:5].cpu().tolist()
        if meta[0] != 0x52505231:
            raise ValueError("not a packed RangeProofList")
        n, u, l, S = meta[1:]
        if n < 0 or l < 0 or S < 0:
            raise ValueError("malformed RangeProofList header")
        o = 5
        if offs is None:
            offs = t[o: o + 2 * n].cpu().clone().view(torch.int64).tolist()
        o += 2 * n
        if cols is None:
            cols = t[o: o + n].cpu().tolist()
        o += n
        has_rp = not (u == 0 and l == 0)
        need = o + 48 * n + ((8 + 8 + 24) * n + 8 * n * l + (8 + 32 + 96) * n * S * l if has_rp and n else 0)
        if need != t.numel():
            raise ValueError(f"packed RangeProofList has {t.numel()} words, header implies {need}")

        def take(rows, width):
            nonlocal o
            v = t[o: o + rows * width].view(rows, width)
            o += rows * width
            return v

        commit = CipherVector(take(n, 24), take(n, 24))
        rpl = RangeProofList(u, l, S, offs, cols, commit)
        if rpl.has_rp and n:
            rpl.challenge, rpl.zr, rpl.D = take(n, 8), take(n, 8), take(n, 24)
            rpl.zphi, rpl.zv = take(n * l, 8), take(n * S * l, 8)
            rpl.V, rpl.A = take(n * S * l, 32), take(n * S * l, 96)
        return rpl

    def to(self, device) -> "RangeProofList":
        mv = lambda t: None if t is None else t.to(device)  # noqa: E731
        return RangeProofList(self.u, self.l, self.S, list(self.offset), list(self.cols), self.commit.to(device),
                              mv(self.challenge), mv(self.zr), mv(self.D), mv(self.zphi), mv(self.zv), mv(self.V),
                              mv(self.A))


# ----------------------------------------------------------------------------- helpers
def to_base(n: int, b: int, l: int) -> list:
    """ToBase (range_proof.go:584): little-endian base-b digits, zero-padded to l.
    Non-positive n gives all-zero digits (reference behaviour)."""
    digits = []
    while n > 0:
        digits.append(n % b)
        n //= b
    while len(digits) < l:
        digits.append(0)
    return digits[:max(l, len(digits))]


def _digits(vals, offs, u: int, l: int) -> np.ndarray:
    """[n, l] base-u digits of m + offset (ToBase per value, vectorised when
    every m + offset fits an unsigned 64-bit word)."""
    try:  # int64 values and offsets: m + offset computed in uint64 without a Python loop
        v = np.asarray(vals, dtype=np.int64).reshape(-1)
        o = np.asarray(offs, dtype=np.int64).reshape(-1)
        ok64 = u >= 2 and v.size > 0 and bool((o >= 0).all() and (v >= -o).all())
    except OverflowError:
        ok64 = False
    if ok64:
        a = v.astype(np.uint64) + o.astype(np.uint64)      # 0 <= m + offset < 2^64: exact
        out = np.empty((a.size, l), dtype=np.int64)
        uu = np.uint64(u)
        for j in range(l):
            out[:, j] = (a % uu).astype(np.int64)
            a //= uu
        return out
    x = [int(v) + int(o) for v, o in zip(vals, offs)]
    return np.array([to_base(v, u, l)[:l] for v in x], dtype=np.int64).reshape(len(x), l)


_pow_cache: dict = {}


def _powers(u: int, l: int, device) -> torch.Tensor:
    """[l, 8] scalars u^j mod r, cached per device."""
    key = (u, l, str(torch.device(device)))
    t = _pow_cache.get(key)
    if t is None:
        t = _pow_cache[key] = bn.publish(bn.scalars_tensor([pow(u, j, O.R) for j in range(l)], device))
    return t


def _rep(t: torch.Tensor, k: int) -> torch.Tensor:
    return t.repeat_interleave(k, dim=0).contiguous()


def _small_scalars(vals, device) -> torch.Tensor:
    a = np.zeros((len(vals), 8), dtype=np.uint32)
    v = np.asarray(vals, dtype=np.int64)
    a[:, 0] = (v & 0xFFFFFFFF).astype(np.uint32)
    a[:, 1] = ((v >> 32) & 0xFFFFFFFF).astype(np.uint32)
    return bn.to_tensor(a, device)


def _challenge_hash(C_aff_bytes: np.ndarray, ysum_bytes: list) -> list:
    """c = SHA3-512(B || C || sum_i y_i) mod r (range_proof.go:350-374)."""
    Bb = O.g1_to_bytes(O.G1_GEN)
    out = []
    for p in range(C_aff_bytes.shape[0]):
        h = hashlib.sha3_512()
        h.update(Bb)
        h.update(C_aff_bytes[p].tobytes())
        h.update(ysum_bytes[p])
        out.append(int.from_bytes(h.digest(), "big") % O.R)
    return out


# ----------------------------------------------------------------------------- prove
def create_range_proofs(batch, sigmat: SigMaterial, P_point, device=None, mode: int = 0) -> list:
    """Batched CreatePredicateRangeProofForAllServ over a CreateProofBatch.
    Returns a list of RangeProofList (one per distinct (u, l)).  ``mode`` 2
    produces the v2 transcript (``SurveyQuery.RangeProofMode``)."""
    device = torch.device(device or batch.cv.device)
    n = len(batch)
    u_arr, l_arr = np.asarray(batch.u, dtype=np.int64), np.asarray(batch.l, dtype=np.int64)
    if n and (u_arr == u_arr[0]).all() and (l_arr == l_arr[0]).all():
        # one (u, l) for the whole batch (every query the simulation runs): no per-item Python loops
        u, l = int(u_arr[0]), int(l_arr[0])
        cols_a = np.asarray(batch.sig_col, dtype=np.int64)
        su = np.asarray(sigmat.u + [0], dtype=np.int64)
        bad_m = (cols_a >= sigmat.n_cols) | (cols_a < 0) | (su[np.clip(cols_a, 0, sigmat.n_cols)] < u)
        if bad_m.any():
            raise ValueError(f"query Ranges base u={u} exceeds the input-validation signatures of column(s) "
                             f"{sorted(set(cols_a[bad_m].tolist()))[:8]} (the CNs signed fewer digits)")
        offs = list(batch.offset) if batch.offset else [0] * n
        return [_prove_group(u, l, batch.values, offs, list(batch.sig_col), batch.r.contiguous(),
                             batch.cv.to(device), sigmat, P_point, device, mode, vals_t=batch.values_t)]
    groups: dict = {}
    for idx in range(len(batch)):
        groups.setdefault((batch.u[idx], batch.l[idx]), []).append(idx)
    out = []
    for (u, l), idxs in groups.items():
        bad = [batch.sig_col[i] for i in idxs
               if batch.sig_col[i] >= sigmat.n_cols or sigmat.u[batch.sig_col[i]] < u]
        if bad:
            raise ValueError(f"query Ranges base u={u} exceeds the input-validation signatures of column(s) "
                             f"{sorted(set(bad))[:8]} (the CNs signed fewer digits)")
        sel = torch.tensor(idxs, dtype=torch.long, device=batch.cv.device)
        cv = CipherVector(batch.cv.K[sel], batch.cv.C[sel])
        vals = [batch.values[i] for i in idxs]
        offs = [batch.offset[i] if batch.offset else 0 for i in idxs]
        cols = [batch.sig_col[i] for i in idxs]
        r = batch.r[sel].contiguous()
        out.append(_prove_group(u, l, vals, offs, cols, r, cv.to(device), sigmat, P_point, device, mode))
    return out


def challenges(C_jac, cols, sigmat: SigMaterial, device, mode: int = 0, D=None, V=None, A=None, S: int = 1,
               l: int = 1) -> torch.Tensor:
    """Fiat-Shamir challenges [n, 8] of a proof list.
    mode < 2: c = SHA3-512(B || C || sum_i y_i) mod r (range_proof.go:350-374),
              on the device (Keccak kernel);
    mode 2  : the v2 transcript, which also binds the commitments:
              c = SHA3-512(B || C || sum_i y_i || D || H(V_p) || H(a_p)) mod r,
              H = SHA-256 over the proof's raw V / a limbs (computed in HBM)."""
    bw, yw = sigmat.challenge_words(device)
    cols_t = bn.h2d(torch.tensor(cols, dtype=torch.int32), device)
    C_aff = nt.g1_to_affine(C_jac.contiguous())
    if mode < 2:
        return nt.rp_challenges(C_aff, bw, yw, cols_t)
    n = C_jac.shape[0]
    hV = nt.sha256_chunks(V.contiguous(), S * l * 128).cpu().numpy().view(np.uint32).astype(">u4").reshape(n, 8)
    hA = nt.sha256_chunks(A.contiguous(), S * l * 384).cpu().numpy().view(np.uint32).astype(">u4").reshape(n, 8)
    Cb = bn.g1_aff_to_bytes(C_aff)
    Db = bn.g1_aff_to_bytes(nt.g1_to_affine(D.contiguous()))
    Bb = O.g1_to_bytes(O.G1_GEN)
    out = []
    for p in range(n):
        h = hashlib.sha3_512()
        h.update(b"drynx_amd/range/v2")
        h.update(Bb)
        h.update(Cb[p].tobytes())
        h.update(sigmat.Ysum_bytes[cols[p]])
        h.update(Db[p].tobytes())
        h.update(hV[p].tobytes())
        h.update(hA[p].tobytes())
        out.append(int.from_bytes(h.digest(), "big") % O.R)
    return bn.scalars_tensor(out, device)


def _digits_dev(vals_t: torch.Tensor, offs: list, u: int, l: int, device, vals: list | None = None):
    """Device [n, l] base-u digits of m + offset (low l digits, as ``_digits``)
    when every power u^j (j < l) and every m + offset fit int64 (|m| < 2^62,
    checked on the host copy ``vals``; 0 <= offset <= 2^62), else None."""
    if u < 2 or u ** (l - 1) >= (1 << 62) or not offs or max(offs) > (1 << 62) or min(offs) < 0:
        return None
    if vals is not None and vals and (max(vals) >= (1 << 62) or min(vals) <= -(1 << 62)):
        return None
    x = vals_t.to(device=device, dtype=torch.int64)
    o = offs[0]
    x = x + (o if offs.count(o) == len(offs) else bn.h2d(torch.tensor(offs, dtype=torch.int64), device))
    pw = bn.h2d(torch.tensor([u ** j for j in range(l)], dtype=torch.int64), device)
    return torch.remainder(torch.div(x.view(-1, 1), pw.view(1, -1), rounding_mode="floor"), u)


def _prove_group(u, l, vals, offs, cols, r, cv, sigmat, P_point, device, mode=0, vals_t=None) -> RangeProofList:
    n = len(vals)
    S = sigmat.S
    rpl = RangeProofList(u, l, S, offs, cols, cv)
    if u == 0 and l == 0:
        return rpl
    r = r.to(device)
    tabB = bn.base_table(device)
    tabP = pk_table(P_point, device).tabP
    # digits of m + offset
    with timers.span("rp.prove.digits"):
        phi_t = _digits_dev(vals_t, offs, u, l, device, vals) if vals_t is not None else None
        phi = _digits(vals, offs, u, l) if phi_t is None else None
    # randomness
    with timers.span("rp.prove.random"):
        s = bn.random_scalars(n * l, device)
        t = bn.random_scalars(n * l, device)
        m = bn.random_scalars(n * l, device)
        v = bn.random_scalars(n * S * l, device)
    # commitments (independent of the challenge):
    # D = (sum_j u^j s_j) B + (sum_j m_j) P
    with timers.span("rp.prove.D"):
        us = nt.fr_dot_rows(s, _powers(u, l, device), n, b_periodic=True)
        msum = nt.fr_dot_rows(m, None, n)
        D = nt.g1_add(nt.g1_fb_mul(tabB, us), nt.g1_fb_mul(tabP, msum))
    # V_ij = v_ij * A_{i, col, phi_j};  a_ij = e(-s_j B, V_ij) e(t_j B, B2)
    cols_t = bn.h2d(torch.tensor(cols, dtype=torch.long), device)
    i_idx = torch.arange(S, device=device)
    if phi_t is None:
        phi_t = bn.h2d(torch.from_numpy(phi), device)
    a_index = ((i_idx.view(1, S, 1) * sigmat.n_cols + cols_t.view(n, 1, 1)) * max(1, sigmat.umax)
               + phi_t.view(n, 1, l)).reshape(-1)
    _, gt_tab = gt_generator_table(device)
    with timers.span("rp.prove.unique"):
        uniq, inv = torch.unique(a_index, return_inverse=True)
        tabs = sigmat.prover_tables(uniq, device, n_items=a_index.numel())
    if tabs is not None:
        # table-driven prover: V = v * A_phi (G2 comb), a = e(B,A_phi)^{-s v} * gT^t (GT combs) --
        # no pairing and no final exponentiation per (value, server, digit)
        g2_tabs, gphi_tabs, slot, wbits = tabs
        tidx = slot.index_select(0, inv).to(torch.int32).contiguous()
        with timers.span("rp.prove.V"):
            V = {4: nt.g2_fb4_mul, 6: nt.g2_gls6_mul, 7: nt.g2_gls8_mul, 8: nt.g2_fb_mul}[wbits](g2_tabs, v, tidx)
        negs_rep = nt.fr_arith(nt.FR_NEG, s).view(n, 1, l, 8).expand(n, S, l, 8).reshape(-1, 8).contiguous()
        e = nt.fr_arith(nt.FR_MUL, negs_rep, v)
        with timers.span("rp.prove.A"):
            A = nt.rp_prove_a_tab(gphi_tabs, tidx, e, t, gt_tab, S, l, wbits)
    else:
        A_sel = sigmat.A.to(device).index_select(0, a_index).contiguous()
        V = nt.g2_mul(A_sel, v)
        # a_ij = FE(ML(-s_j B, V_ij)) * gT^{t_j}
        negsB = nt.g1_to_affine(nt.g1_fb_mul(tabB, nt.fr_arith(nt.FR_NEG, s)))
        A = nt.rp_prove_a(negsB, V, t, gt_tab, S, l)
    # Fiat-Shamir challenge per value
    with timers.span("rp.prove.challenge"):
        c = challenges(cv.C, cols, sigmat, device, mode, D, V, A, S, l)
    # responses: Zphi_j = s_j - c phi_j ; Zr = sum m - c r ; Zv_ij = t_j - c v_ij
    if phi is None:
        phi_sc = torch.zeros((n * l, 8), dtype=torch.int32, device=device)
        phi_sc[:, 0] = phi_t.reshape(-1).to(torch.int32)              # 0 <= phi < u < 2^31
    else:
        phi_sc = _small_scalars(phi.reshape(-1), device)
    with timers.span("rp.prove.responses"):
        zphi = nt.fr_arith(nt.FR_SUB, s, nt.fr_arith(nt.FR_MUL, _rep(c, l), phi_sc))
        zr = nt.fr_arith(nt.FR_SUB, msum, nt.fr_arith(nt.FR_MUL, c, r))
        t_rep = t.view(n, 1, l, 8).expand(n, S, l, 8).reshape(-1, 8).contiguous()
        zv = nt.fr_arith(nt.FR_SUB, t_rep, nt.fr_arith(nt.FR_MUL, _rep(c, S * l), v))
    rpl.challenge, rpl.zr, rpl.D, rpl.zphi, rpl.zv, rpl.V, rpl.A = c, zr, D, zphi, zv, V, A
    return rpl


# ----------------------------------------------------------------------------- verify
def _rand64(n, device, bits: int = 64) -> torch.Tensor:
    """Uniform ``bits``-bit batch weights from the ChaCha20 CSPRNG (device or
    host path), unknown to the prover."""
    from ..crypto.coins import mask_bits

    return mask_bits(bn.random_scalars(n, device), bits)


def _gt_in_subgroup(g: torch.Tensor) -> bool:
    """Host test that cyclotomic elements are in GT (order r): g^p == g^(6u^2)
    (p = 6u^2 mod r for BN curves; Scott's membership test)."""
    return all(_gt_in_subgroup_each(g))


def _gt_in_subgroup_each(g: torch.Tensor) -> list:
    """``_gt_in_subgroup`` of every row of [k, 96] -> [bool] (one host batch:
    x^p by a Frobenius map against x^(6u^2) by two cyclotomic u-ladders; the
    rows are products of validated cyclotomic a_ij)."""
    return [bool(v) for v in nt.gt_membership(g.cpu().contiguous()).tolist()]


class RangeInvalid(list):
    """Verdict of a segmented batch rejected at decoding: per segment, whether
    all its proofs decode (the batch equations were not evaluated; the valid
    segments need a batch of their own)."""


def validate_list(r: RangeProofList, mode: int = 0, subgroup: bool | None = None, lazy: bool = False,
                  per_proof: bool = False):
    """Decoding checks of a (raw-limb or kyber-layout) proof list before any
    arithmetic on it: every coordinate below p and every scalar below r; the
    commitment (K, C) and D on G1; V in G2 (``subgroup``, default: mode >= 1)
    or only on the twist; every a_ij non-zero and in the cyclotomic subgroup.
    The prime-order part of a_ij is enforced by the batch equation plus each
    VN's independent random combination tested in GT.  ``lazy``: return the
    verdict as a device bool (no host sync); ``per_proof``: a bool per proof."""
    if subgroup is None:
        subgroup = mode >= 1
    fp = lambda t: nt.limbs_canonical(t.reshape(-1, 8))  # noqa: E731
    fr = lambda t: nt.limbs_canonical(t.reshape(-1, 8), fr=True)  # noqa: E731
    flags = [fp(r.commit.K), fp(r.commit.C), nt.g1j_on_curve(r.commit.K), nt.g1j_on_curve(r.commit.C)]
    if r.has_rp and len(r):
        flags += [fp(r.D), nt.g1j_on_curve(r.D), fr(r.challenge), fr(r.zr), fr(r.zphi), fr(r.zv), fp(r.V), fp(r.A),
                  nt.g2_subgroup(r.V) if subgroup else nt.g2_on_curve(r.V), nt.gt_cyclotomic(r.A)]
    # every array is proof-major with a fixed number of rows per proof: one
    # per-proof AND of all of them (nt.rows_all: a wavefront per proof)
    n = len(r)
    ok = nt.rows_all(flags, n).bool() if n else torch.ones((0,), dtype=torch.bool, device=r.commit.K.device)
    if per_proof:
        return ok if lazy else ok.tolist()
    ok = ok.all()
    return ok if lazy else bool(ok)


def verify_range_proof_list(rpl: RangeProofList, sigmat: SigMaterial, P_point, threshold: float = 1.0,
                            device=None, mode: int = 0, coins=None) -> bool:
    """RangeProofListVerification: verifies the first ceil(threshold * n)
    proofs of the list (reference sampling semantics) as ONE batch.
    ``mode`` (``SurveyQuery.RangeProofMode``): 0 trusts the proof's challenge
    like range_proof.go:504-565; >= 1 recomputes it (v1 / v2 transcript) and
    requires every V_ij in G2."""
    if not rpl.has_rp:
        return True
    k = int(math.ceil(threshold * len(rpl)))
    if k == 0:
        return True
    r = rpl if k == len(rpl) else _slice(rpl, k)
    return verify_range_proof_list_multi(r, sigmat, P_point, 1, device, mode, coins=[coins])[0]


def verify_range_proof_list_multi(r: RangeProofList, sigmat: SigMaterial, P_point, n_vn: int = 1, device=None,
                                  mode: int = 0, coins: list | None = None, segs: list | None = None) -> list:
    """``n_vn`` independent batch verifications of one proof list -- one per
    verifying node hosted on this rank, each with its own random weights
    drawn from its own ``coins[v]`` (crypto/coins.py; fresh CSPRNG output
    when None).

    Per VN v the l*S pairing equations of all n proofs are combined with
    uniform 64-bit weights rho_v, and the n D-equations with w_v:
      FE(prod_it ML(rho_it (Zphi_j B - c y_i), V_it)) * prod_it a_it^rho_it
          == gT^(sum rho Zv)                                  (one final exp)
      sum w (c C') + (sum w Zr) P + (sum w z) B == sum w D       (one MSM)
    plus GT membership of the a_it: each VN's own independent 40-bit
    combination gamma_v.  What does not depend on the weights -- decoding
    checks, the strict-mode
    challenge and G2 checks, Zphi*B, c*y_i and their differences -- is
    computed once for the co-hosted VNs.  On a GPU the VNs' Miller folds are
    queued back to back (no host round trip between them) while the
    bucket-method MSM / multi-exponentiations run on a side stream; the
    closing single-element work (final exponentiations, Horner steps) runs
    on the host, where one core beats one GPU lane.  -> [bool] per VN.

    ``segs`` (proof counts summing to len(r): the batch's per-request
    slices) asks for attribution: -> per VN a [bool] per segment, None when
    a failed batch cannot be attributed, or a
    ``RangeInvalid`` (per segment: decodes) when some proofs do not decode.  The U side is then laid out per segment
    (each segment's U_q start whole accumulation workgroups, so each has its
    own Miller partial products -- no extra pairing work), and only a VN
    whose batch FAILS pays a second, segment-grouped pass over the cheap
    sides (R MSM, multi-exponentiation, D-check, exponent sums) with the same
    weights: blame costs ~one VN's MSMs, not a bisection of re-verifications."""
    nseg = len(segs) if segs else 1
    if segs is not None:
        assert sum(segs) == len(r) and all(c > 0 for c in segs)
    if not r.has_rp or len(r) == 0:
        return [True] * n_vn if segs is None else [[True] * nseg for _ in range(n_vn)]
    fail = [False] * n_vn if segs is None else [None] * n_vn
    device = torch.device(device or r.commit.device)
    r = r.to(device)
    n, l, S, u = len(r), r.l, r.S, r.u
    if r.zphi.shape[0] != n * l or r.zv.shape[0] != n * S * l or r.V.shape[0] != n * S * l \
            or r.A.shape[0] != n * S * l or r.challenge.shape[0] != n:
        return fail
    # pairing side regrouped by bilinearity: one G2 MSM and n*S L-point
    # combinations per VN, n*S + 1 Miller loops (``_msm_queue``)
    dmode = os.environ.get("DRYNX_DCHECK", "auto")
    ddirect = dmode == "direct" or (dmode == "auto" and device.type == "cuda" and n * n_vn <= _DCHECK_DIRECT_MAX)
    cC = ev_cC = ev_valid = table = None
    if device.type == "cuda":
        # the U side's joint tables depend on V alone: first on this stream, so
        # the U chain (the critical path of a small batch) starts at once
        with timers.span("rp.u.joint_table"):
            table = nt.g2_joint_table(r.V)
    with timers.span("rp.verify.validate"):
        # On a GPU the checks run on their own stream, filling the gaps the
        # verifier's host-side plans leave, and are read back with the
        # verdicts (work done meanwhile on invalid data is discarded)
        vstream = _val_stream(device) if device.type == "cuda" else None
        pp = segs is not None
        chk = None
        if vstream is not None:
            vstream.wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(vstream):
                valid = validate_list(r, mode, lazy=True, per_proof=pp)
                ev_valid = torch.cuda.Event()
                ev_valid.record(vstream)                      # the weight mask waits for this, not for c C'
                if ddirect:  # c C' per proof, weight-free (undecodable rows are masked out later)
                    cC = nt.g1_mul(r.commit.C.contiguous() if not any(r.offset) else
                                   nt.g1_add(r.commit.C, nt.g1_fb_mul_i64(
                                       bn.base_table(device), bn.h2d(torch.tensor(r.offset, dtype=torch.int64),
                                                                     device))),
                                   r.challenge.contiguous())
                    ev_cC = torch.cuda.Event()
                    ev_cC.record(vstream)
        else:
            valid = validate_list(r, mode, lazy=True, per_proof=pp)
            if not bool(valid.all()) and segs is None:
                return _invalid(valid, segs, n_vn)
    if mode >= 1:
        with timers.span("rp.verify.challenge"):
            ch_ok = (challenges(r.commit.C, r.cols, sigmat, device, mode, r.D, r.V, r.A, S, l)
                     == r.challenge).all(dim=1)
            if segs is None:
                if not bool(ch_ok.all()):
                    return _invalid(ch_ok, segs, n_vn)
            else:
                chk = ch_ok                    # a wrong challenge fails its own segment (attributed below)
    tabB = bn.base_table(device)
    # --- per-VN weights (each from its own coins): every VN's bucket plans in
    # ONE host sync each.  Drawn before the weight-free inputs: on a GPU the U
    # combinations (queue stream) and the R MSM (aux stream) need only these
    # and the joint tables, so both chains start before the host has issued
    # the inputs' small launches (c y_i, sum Zphi u^j, C')
    G, m = n_vn, n * S * l
    cl = list(coins) if coins is not None else [None] * G
    cl += [None] * (G - len(cl))

    def _cat_draw(fn):
        return torch.cat([fn(c) for c in cl]) if G > 1 else fn(cl[0])

    _sw = timers.span("rp.verify.weights")
    _sw.__enter__()
    # D-equation weights, GLV-shaped like rho (a + b lambda, 32-bit halves:
    # the same 2^-64 soundness as uniform 64-bit weights), so the D-check can
    # run as 32-doubling GLV ladders with no bucket plan
    wpairs = [c.glv(n, device) if c is not None else nt.glv_weights(n, device) for c in cl]
    wab_all = torch.cat([p_[0] for p_ in wpairs]) if G > 1 else wpairs[0][0]
    w_all = torch.cat([p_[1] for p_ in wpairs]) if G > 1 else wpairs[0][1]
    # pairing-equation weights: rho = a + b lambda (GLV, a and b 32-bit: 2^64
    # distinct residues, so the same 2^-64 soundness as uniform 64-bit weights;
    # csrc/kernels/dx_glv.hip)
    pairs = [c.glv(m, device) if c is not None else nt.glv_weights(m, device) for c in cl]
    ab_all = torch.cat([p_[0] for p_ in pairs]) if G > 1 else pairs[0][0]
    rho_all = torch.cat([p_[1] for p_ in pairs]) if G > 1 else pairs[0][1]
    # GT-membership combinations: one independent 40-bit gamma set PER VN
    gb = _gamma_bits()
    gam_all = _cat_draw(lambda c: c.bits(m, device, gb) if c is not None else _rand64(m, device, gb))
    # attribution: undecodable proofs (and, mode >= 1, wrong challenges) get
    # ZERO weights -- every weighted sum then runs over the decodable proofs
    # only (their U_q and -c y_i become infinity, as the fold's padding), so
    # one bad payload costs no second pass: the batch verdict IS the verdict
    # of the decodable segments
    masked = segs is not None
    vm = None
    if masked:
        if ev_valid is not None:
            torch.cuda.current_stream(device).wait_event(ev_valid)
        vm = (valid if chk is None else valid & chk).to(torch.int32)
        mi = vm.repeat_interleave(S * l).view(1, m, 1)
        w_all = (w_all.view(G, n, 8) * vm.view(1, n, 1)).view(G * n, 8)
        wab_all = (wab_all.view(G, n, 2) * vm.view(1, n, 1)).view(G * n, 2)
        ab_all = (ab_all.view(G, m, 2) * mi).view(G * m, 2)
        rho_all = (rho_all.view(G, m, 8) * mi).view(G * m, 8)
        gam_all = (gam_all.view(G, m, 8) * mi).view(G * m, 8)
    _sw.__exit__(None, None, None)
    vns = [{"rho": rho_all[v * m:(v + 1) * m], "ab": ab_all[v * m:(v + 1) * m]} for v in range(G)]
    timers.count("rp.verify.items", G * m)
    me_groups = ((2 * m, 32),) * G + ((m, gb),) * G
    # windows by cost (nt.me_window): 16 bits for a 1-GPU inbox, 11 for a pool
    # slice; the host keeps bytes (fewer buckets for its serial products)
    wc_ = nt.me_window(me_groups) if device.type == "cuda" else (5, 8)
    aux = _aux_stream(device) if device.type == "cuda" else None
    meta = (G, m, S, l, gb, tuple(wc_), _r_window(m, G))
    ev_u = ev_r = None
    if aux is not None:
        # the R MSM needs only V, Zphi and the weights: queued on the aux stream now
        ready_w = torch.cuda.Event()
        ready_w.record(torch.cuda.current_stream(device))
        aux.wait_event(ready_w)
        with timers.span("rp.verify.passes"), torch.cuda.stream(aux):
            S_R, hR = _pass_r(r.V, r.zphi, rho_all, meta)
            ev_r = torch.cuda.Event()                                   # the R MSM is queued
            ev_r.record(aux)
    # --- shared, weight-free inputs: the fold's points c y_i (on a GPU issued
    # by _msm_queue after the U combinations, on the U stream), and C' and
    # sum_j Zphi_j u^j for the D-check and the exponent sums (on the aux
    # stream, before the multi-exponentiation: nothing there waits for the U side)
    inp = {}

    def _inputs():
        with timers.span("rp.verify.inputs"):
            cols_t = bn.h2d(torch.tensor(r.cols, dtype=torch.long), device)
            y_idx = (torch.arange(S, device=device).view(1, S) * sigmat.n_cols + cols_t.view(n, 1)).reshape(-1)
            ytabs = sigmat.y_tables(device)
            if ytabs is not None:                                              # c * y_i as fixed-base mults
                Y = nt.g1_fb_mul_idx(ytabs[0], ytabs[1].index_select(0, y_idx).contiguous(), _rep(r.challenge, S))
            else:
                Y = nt.g1_mul(sigmat.y_jac.to(device).index_select(0, y_idx).contiguous(),
                              _rep(r.challenge, S))                             # [n*S]
            if vm is not None:
                Y = Y.clone()
                Y[:, 16:] *= vm.repeat_interleave(S).view(-1, 1)                # Z = 0: -c y_i at infinity
        inp["Y"] = Y
        return Y

    def _zcp():
        Cp = r.commit.C                                                        # C' = C + offset*B
        if any(r.offset):
            Cp = nt.g1_add(Cp, nt.g1_fb_mul_i64(tabB, bn.h2d(torch.tensor(r.offset, dtype=torch.int64), device)))
        return Cp, nt.fr_dot_rows(r.zphi, _powers(u, l, device), n, b_periodic=True)   # sum_j Zphi_j u^j

    # GPU: the U side on this stream (its chain of Miller-loop kernels is the
    # critical path of a small batch), the R MSM (above), the
    # multi-exponentiation and the D-check on the aux stream.  (Launching the R
    # MSM before the U side measured neutral on the pool parts and +2.5 ms on
    # the 1-GPU query: the two chains only slow each other down on the shared
    # CUs; here both are queued before the inputs.)
    if aux is not None:
        with timers.span("rp.verify.msm_queue"):
            msq = _msm_queue(_inputs, r.V, ab_all, G, n, S, l, vstream, segs, table)
            for v, uok in zip(vns, msq["u_ok"]):
                v["u_ok"] = uok
        ev_u = torch.cuda.Event()                                       # the U side's fold is queued
        ev_u.record(torch.cuda.current_stream(device))
    else:
        _inputs()
    with timers.span("rp.verify.passes"), (torch.cuda.stream(aux) if aux is not None else _nullctx()):
        Cp, z = _zcp()
        if not ddirect:
            dpts = torch.cat([Cp.contiguous(), r.D.contiguous()]).repeat(G, 1)
            wc = nt.fr_arith(nt.FR_MUL, w_all, r.challenge)
            dsc = torch.stack([wc.view(G, n, 8), w_all.view(G, n, 8)], 1).reshape(-1, 8).contiguous()
        if aux is None:
            S_R, hR = _pass_r(r.V, r.zphi, rho_all, meta)
        A2, mexp, e_all, dfull = _pass_me(r.A, ab_all, gam_all, rho_all, r.zv, w_all, r.zr, z, meta)
        with timers.span("rp.run.D"):
            if ddirect:
                if cC is None:                                                 # host path
                    cC = nt.g1_mul(Cp.contiguous(), r.challenge.contiguous())
                elif ev_cC is not None:
                    torch.cuda.current_stream(device).wait_event(ev_cC)
                pts = torch.stack([cC, r.D], 1).unsqueeze(1).expand(n, G, 2, 24).reshape(-1, 24)
                abs_ = wab_all.view(G, n, 2).permute(1, 0, 2).unsqueeze(2).expand(n, G, 2, 2).reshape(-1, 2)
                # item-major [n, 2G]: group v * 2 + which, summed over the proofs
                dcheck = nt.g1_sum(nt.g1_mul_glv(pts.contiguous(), abs_.contiguous()).view(n, 2 * G, 24))
            else:
                dcheck = nt.g1_msm_device(dpts, dsc, n, ((n, 254),) * (2 * G))     # group = row // n
    if aux is None:  # host: the U side after the passes
        msq = _msm_queue(inp["Y"], r.V, ab_all, G, n, S, l, None, segs)
        for v, uok in zip(vns, msq["u_ok"]):
            v["u_ok"] = uok
    useg = fR = None
    with timers.span("rp.verify.multiexp"):
        if aux is not None:
            run_idle_tasks()  # host work queued by the caller, in the GPU's busiest window
            # the host tails of the R side (Horner, ML(B, R)) and of the U side
            # (per-segment products) as soon as their device chains are done,
            # while the multi-exponentiation and the D-check still run
            ev_r.synchronize()
            with timers.span("rp.verify.r_tail"):
                fR, rok = _msm_r_miller(hR, S_R)
            ev_u.synchronize()
            with timers.span("rp.verify.u_tail"):
                useg = _seg_products(msq)                              # [G, nseg, 96] host
            aux.synchronize()                                          # aux results are read on this stream/host
        GG = nt.multi_exp_grouped_finish(mexp)                         # [2G, 96]: prod a^rho_v, prod a^gamma_v
        D_all = dcheck.cpu() if ddirect else nt.g1_msm_finish(dcheck)  # [2G, 24]
        for h_ in (mexp, hR) if ddirect else (mexp, hR, dcheck):
            nt.check_overflow(h_)
        e_all, dfull = e_all.cpu(), dfull.cpu()
    with timers.span("rp.verify.fold_wait"):
        if useg is None:
            useg = _seg_products(msq)                                  # [G, nseg, 96] host
        for k_, v in enumerate(vns):
            v["F"] = nt.gt_prod(useg[k_].view(nseg, 1, 96), chunk=64).view(1, 96)
        if fR is None:
            fR, rok = _msm_r_miller(hR, S_R)
        for v, f, ok in zip(vns, fR, rok):
            v["F"], v["r_ok"] = nt.gt_mul(v["F"], f.view(1, 96)), ok
    for k, v in enumerate(vns):
        v.update(G=GG[k: k + 1], dfull=dfull[k], e=e_all[k: k + 1], dcheck=D_all[2 * k: 2 * k + 2])
    if vstream is not None:
        vstream.synchronize()
    if chk is not None:
        valid = valid & chk
    if vstream is not None:
        if not bool(valid.all()) and segs is None:
            return _invalid(valid, segs, n_vn)
    out = []
    # prime-order part of the a_ij: each VN's own independent 40-bit
    # combination in GT (the smallest prime factor of the cyclotomic cofactor
    # is ~2^38.8: a non-GT component survives the batch equation AND this test
    # with probability ~2^-77)
    m_oks = _gt_in_subgroup_each(GG[G: 2 * G])
    _, gt_tab = gt_generator_table("cpu")
    PB_base = bn.g1_jac_tensor([P_point, O.G1_GEN], "cpu")
    with timers.span("rp.verify.final_exp"):
        # every VN's final exponentiation in one host batch (one core each)
        fe = nt.final_exp(torch.cat([v["F"].cpu().view(1, 96) for v in vns]).contiguous())
    for k_, v in enumerate(vns):
        with timers.span("rp.verify.finish"):
            G0 = v["dcheck"]
            PB = nt.g1_mul(PB_base, v["dfull"])
            v["dl"] = nt.g1_sum(torch.stack([G0[0:1], PB[0:1], PB[1:2]]))
            d_ok = bool(nt.g1_eq(v["dl"], G0[1:2])[0])
            v["lhs"] = lhs = nt.gt_mul(fe[k_: k_ + 1].contiguous(), v["G"].cpu())
            eq_ok = bool(nt.gt_eq(lhs, nt.gt_fb_pow(gt_tab, v["e"].cpu())).all())
        # regrouped ("msm") check: the U_q and R of this VN must lie in G2 --
        # then their torsion parts (V_it off G2 by a cofactor component) cancel
        # and the checked equation is the one of the proof's G2 projection,
        # where the pairing is bilinear and the regrouping exact
        g2_ok = bool(v.get("u_ok", True)) and bool(v.get("r_ok", True))
        out.append(d_ok and m_oks[len(out)] and eq_ok and g2_ok)
        if not out[-1]:
            log.warning(f"range batch of {n} proofs failed for verifier {len(out) - 1}: D-check {d_ok}, "
                        f"GT membership {m_oks[len(out) - 1]}, pairing equation {eq_ok}, "
                        f"U in G2 {bool(v.get('u_ok', True))}, R in G2 {bool(v.get('r_ok', True))}")
    if segs is None:
        return out
    # attribution: a passing batch clears every segment; a failing one gets
    # the segment-grouped second pass.  Undecodable proofs fail their own
    # segments only: every per-segment quantity (U_q, the fold blocks, R_s,
    # prod a^rho, the D-check) involves that segment's data alone
    seg_valid = None if bool(valid.all()) else _seg_all(valid.view(1, -1), segs, valid.device).view(-1).tolist()
    # masked weights: a passing batch clears every decodable segment
    redo = [k_ for k_ in range(G) if not out[k_] or (seg_valid is not None and not masked)]
    res = [([True] * nseg if seg_valid is None else list(seg_valid)) if ok else None for ok in out]
    if redo:
        with timers.span("rp.verify.segments"):
            x = dict(A2=A2, rho=rho_all, ab=ab_all, gam=gam_all, w=w_all, Cp=Cp, z=z, useg=useg, u_seg=msq["u_seg"],
                     # the segment pass keeps host-planned 11-bit windows (its groups are
                     # (VN, segment) pairs: 16-bit windows would mean millions of buckets)
                     PB_base=PB_base, gt_tab=gt_tab, wc=(4, 11) if device.type == "cuda" else wc_, G=G,
                     # undecodable proofs in an UNMASKED batch: the first pass's GT
                     # combination included a_ij not known to be cyclotomic, so it
                     # bounds nothing -- every segment then gets its own combination
                     m_first=m_oks if seg_valid is None or masked else [False] * G,
                     tot=dict(lhs=[v.get("lhs") for v in vns], e=e_all, GGgam=GG[G: 2 * G],
                              dl=[v.get("dl") for v in vns], dr=[v["dcheck"][1:2] for v in vns],
                              r_ok=[bool(v.get("r_ok", True)) for v in vns]))
            if masked or seg_valid is None:
                per = _attribute_hinted(r, segs, redo, x)
            else:
                per = _segment_pass(r, segs, redo, x)
        for k_ in redo:
            if seg_valid is not None:
                per_k = [a and b for a, b in zip(per[k_], seg_valid)]
                # masked: the failing batch held decodable proofs only -- a pass
                # of every decodable segment explains nothing (the caller bisects)
                res[k_] = None if masked and per_k == seg_valid else per_k
            else:
                res[k_] = per[k_] if not all(per[k_]) else None  # nothing attributable: the caller bisects
    return res


_idle = threading.local()


class Deferred:
    """A host computation run once, at the first of ``run()`` (e.g. from
    ``run_idle_tasks`` while the verifier waits for its device work) or
    ``result()``."""

    def __init__(self, fn):
        self.fn, self.done, self.value = fn, False, None

    def run(self):
        if not self.done:
            self.value, self.done = self.fn(), True

    def result(self):
        self.run()
        return self.value


def add_idle_task(d: Deferred) -> Deferred:
    """Queue host work for this thread's next verifier wait: the batch
    verifier runs it right before it blocks on the device (its passes then
    keep the GPU busy for milliseconds while the host is idle), instead of a
    second thread contending for the GIL with the verifier's host work."""
    if not hasattr(_idle, "tasks"):
        _idle.tasks = []
    _idle.tasks.append(d)
    return d


def run_idle_tasks():
    tasks = getattr(_idle, "tasks", None)
    while tasks:
        tasks.pop(0).run()


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


_SHAPE_INDEX: dict = {}
_SHAPE_INDEX_MAX = 16


def _shape_index(key, device, fn, n: int) -> torch.Tensor:
    """``fn(arange(n))`` -- an index that depends on the batch shape only
    (item -> Zphi row, multi-exponentiation entry -> group) -- built once per
    shape and device: a query's ~9M-entry arange and its elementwise glue ran
    on every verification pass (profiles/r6/cost/span_kernels.txt).
    Published (ready on every stream) when built; every reading stream is
    recorded on it and the cache drains the device before it drops entries,
    as the plan layouts and the key and signature caches do."""
    k = (key, str(torch.device(device)))
    t = _SHAPE_INDEX.get(k)
    if t is None:
        if len(_SHAPE_INDEX) >= _SHAPE_INDEX_MAX:
            if torch.device(device).type == "cuda":
                torch.cuda.synchronize(device)
            _SHAPE_INDEX.clear()
        t = _SHAPE_INDEX[k] = bn.publish(fn(torch.arange(n, device=device)).contiguous())
    if t.is_cuda:
        t.record_stream(torch.cuda.current_stream(t.device))  # a later drop waits for this reader
    return t


def _pass_r(V, zphi, rho, meta):
    """R = sum_it (rho_it Zphi_(p, j)) V_it per VN: the G2 Pippenger MSM with a
    device plan, queued on the current stream (no host sync) -> (S_R, hR)."""
    G, m, S, l, gb, wc, cR = meta
    zi = _shape_index(("zphi", m, S, l), V.device,
                      lambda it: (it // (S * l)) * l + it % l, m)        # item -> its Zphi row
    s_r = nt.fr_arith(nt.FR_MUL, rho, zphi.index_select(0, zi).contiguous())
    with timers.span("rp.run.R"):
        return nt.g2_msm_device(V, s_r, m, ((m, 254),) * G, c=cR)


def _pass_me(A, ab, gam, rho, zv, w, zr, z, meta):
    """The GT multi-exponentiation over (A, frob^8 A) with the GLV halves of
    rho (groups 0..G-1) and each VN's 40-bit membership combination (G..2G-1),
    and the Fr exponent sums, on the current stream -> (A2, mexp, e_all, dfull)."""
    G, m, S, l, gb, wc, cR = meta
    dev = A.device
    with timers.span("rp.frob8"):  # (A, frob^8 A) stacked: the Frobenius image written in place
        A2 = torch.empty((2 * m, 96), dtype=torch.int32, device=dev)
        A2[:m].copy_(A)
        nt.gt_frob8(A.contiguous(), out=A2[m:])
    abv = ab.view(G, m, 2)
    k = torch.zeros((3 * G * m, 8), dtype=torch.int32, device=dev)
    kr = k[: 2 * G * m].view(G, 2 * m, 8)
    kr[:, :m, 0] = abv[:, :, 0]
    kr[:, m:, 0] = abv[:, :, 1]
    k[2 * G * m:] = gam
    mgrp = _shape_index(("mgrp", G, m), dev,                         # entry -> group
                        lambda e: torch.where(e < 2 * G * m, e // (2 * m), G + (e - 2 * G * m) // m).to(torch.int32),
                        3 * G * m)
    with timers.span("rp.run.ME"):
        mexp = nt.multi_exp_device(A2, k, mgrp, ((2 * m, 32),) * G + ((m, gb),) * G, wc[0], wc[1],
                                   item_split=(2 * G * m, m))
    e_all = nt.fr_dot_rows(rho, zv, G, b_periodic=True)                                 # sum rho Zv per VN
    dfull = torch.stack([nt.fr_dot_rows(w, zr, G, b_periodic=True),
                         nt.fr_dot_rows(w, z, G, b_periodic=True)], 1)                   # [G, 2, 8]
    return A2, mexp, e_all, dfull


_DCHECK_DIRECT_MAX = 16384  # proofs x VNs up to which the D-check runs without a bucket plan


def _r_window(m: int, G: int) -> int:
    """Window bits of the R MSM: ~(bucket additions per entry) x entries +
    (weight and window-sum additions per bucket) x buckets, over 254-bit
    scalars -- 13 bits for a 1-GPU inbox (1M items per VN), ~11 for a pool
    helper's 1/8 slice (a fixed 13-bit plan would weigh 491k mostly-empty
    buckets there)."""
    return min(range(8, 14), key=lambda c: -(-254 // c) * (m + 8 * (1 << c)))


def _msm_queue(Y, V, ab_all, G: int, n: int, S: int, L: int, vstream=None, segs: list | None = None,
               table=None) -> dict:
    """Verifier mode "msm", the U side (no host sync; csrc/kernels/dx_rpmsm.hip):
    the pairing side of G verifiers' batches regrouped by bilinearity,
        prod_it ML(rho_it (Zphi_pj B - Y_pi), V_it)
          ~ ML(B, R_v) * prod_q ML(-Y_q, U_vq)         (equal after the final exp)
    with U_vq = sum_j rho_(q,j) V_(q,j) (q = p*S + i; a joint 2-bit-window
    ladder over the 15-entry per-V table shared by the VNs) and R_v the
    Pippenger G2 MSM of ``_msm_plan`` (queued separately: ``nt.g2_msm_run``,
    finished by ``_msm_r_miller``).  GPU: the U's of all VNs form one list
    (VN-major; with ``segs``, each segment's U's start a whole accumulation
    workgroup) that the normalised fold kernels pair with uv(-Y_q) -> per-
    workgroup partial products ("fb"), reduced per (VN, segment) by
    ``_seg_products``; host: per-item Miller loops over the same pairs.
    "u_seg": [G, n_segments] exact G2 membership of every segment's U's.
    ``Y`` may be a callable returning it (issued after the U combinations)."""
    dev = V.device
    nq = n * S
    nseg = len(segs) if segs else 1
    qoff = np.cumsum([0] + [c * S for c in segs]) if segs else np.array([0, nq])
    cq = np.diff(qoff)
    if table is None:
        with timers.span("rp.u.joint_table"):
            table = nt.g2_joint_table(V)
    out = {"G": G}
    if dev.type == "cuda":
        if nseg == 1:
            K = fold_k(G * (nq + 1))
            rows = 64 * K
            pad = -(-(nq + 1) // rows) * rows
        else:
            K = fold_k(G * nq)
            rows = 64 * K
            ac = -(-cq // rows) * rows                              # segments start whole workgroups
            segbase = np.cumsum(ac) - ac
            pad = int(ac.sum())
        period = -(-(G * pad) // (rows * nt.FOLD_P_ALIGN)) * (rows * nt.FOLD_P_ALIGN)
        # a small batch (a pool slice) folds on three lanes per item over the
        # raw line coefficients and affine points (-Y); a large one keeps the
        # one-lane accumulation over normalised lines and (x/y, 1/y) points
        # (the three-lane fold at the 1-GPU size: no faster, profiles/r6/ab/)
        coop = K == 1 and G * pad <= _COOP_MAX_ITEMS
        Uall = torch.zeros((G * pad, 32), dtype=torch.int32, device=dev)
        UV = torch.zeros((period, 16), dtype=torch.int32, device=dev)
        pos = None
        if nseg > 1:
            # row of (VN v, group q) in the fold layout (segments start whole
            # workgroups): host-known, one upload before the U kernels -- no
            # index glue between the combinations and the fold's coefficients
            qseg = np.repeat(np.arange(nseg), cq)
            qpos = segbase[qseg] + np.arange(nq) - qoff[:-1][qseg]
            pos = _h2d((np.arange(G).reshape(G, 1) * pad + qpos.reshape(1, nq)).reshape(-1).astype(np.int64), dev)
        with timers.span("rp.u.joint"):
            nt.rp_u_joint(table, ab_all, nq, G, L, Uall, pad, pos)
        # G2 membership of every U (exact test), on the validation stream beside the fold
        cur = torch.cuda.current_stream(dev)
        vs = vstream if vstream is not None else cur
        vs.wait_stream(cur)
        with torch.cuda.stream(vs):
            # every read of the flags stays on the validation stream: a reduction
            # queued on `cur` would race the membership kernels (read before they
            # finish); the caller synchronises `vs` before looking at the verdicts
            flags = nt.g2_subgroup(Uall)
            fl = (flags.view(G, pad)[:, :nq] if pos is None else flags.index_select(0, pos).view(G, nq)).bool()
            out["u_seg"] = _seg_all(fl, cq, dev)
            out["u_ok"] = list(out["u_seg"].all(dim=1).unbind(0))
        Uall.record_stream(vs)
        if pos is not None:
            pos.record_stream(vs)
        # the points of the fold (affine -Y_q, or uv(-Y_q) for the normalised
        # lines), after the U combinations are queued (``Y`` may be the
        # callable that issues their inputs)
        if callable(Y):
            Y = Y()
        if coop:  # affine -Y_q, the same for every VN
            negY = nt.g1_to_affine(nt.g1_add(bn.g1_infinity_jac(nq, dev), Y.contiguous(), subtract=True))
        elif nseg > 1:  # uv(-Y_q) is the same for every VN: computed once, copied per VN below
            UVd = torch.zeros((nq + 1, 16), dtype=torch.int32, device=dev)
            nt.rp_msm_uv(Y, UVd, nq, 1, nq + 1)
            negY = UVd[:nq]
        if nseg == 1:
            if coop:
                UV[: G * pad].view(G, pad, 16)[:, :nq] = negY
            else:
                nt.rp_msm_uv(Y, UV, nq, G, pad)
        else:
            UV.index_copy_(0, pos, negY.repeat(G, 1))
        with timers.span("rp.u.fold"):
            if coop:
                out["fb"] = nt.rp_fold_accum_coop_raw(nt.rp_fold_coeffs(Uall), UV, Uall, period, 1)
            else:
                out["fb"] = nt.rp_fold_accum_n(nt.rp_fold_ncoeffs(Uall), UV, Uall, period, 1, K)
        out["blk"] = pad // rows
        out["sb"] = [0] if nseg == 1 else (segbase // rows).tolist()
        out["nb"] = [pad // rows] if nseg == 1 else (ac // rows).tolist()
    else:
        if callable(Y):
            Y = Y()
        Uall = torch.zeros((G * nq, 32), dtype=torch.int32, device=dev)
        nt.rp_u_joint(table, ab_all, nq, G, L, Uall, nq)
        out["u_seg"] = _seg_all(nt.g2_subgroup(Uall).view(G, nq).bool(), cq, dev)
        out["u_ok"] = [bool(x) for x in out["u_seg"].all(dim=1).tolist()]
        negY = nt.g1_to_affine(nt.g1_add(bn.g1_infinity_jac(nq, dev), Y.contiguous(), subtract=True))
        out["fb"] = torch.cat([nt.miller_loop(negY, Uall[v * nq:(v + 1) * nq].contiguous()) for v in range(G)])
        out["blk"], out["sb"], out["nb"] = nq, qoff[:-1].tolist(), cq.tolist()
    return out


def _h2d(a, dev) -> torch.Tensor:
    """A small host array (list / numpy) on ``dev`` through pinned memory: a
    pageable copy would block this thread until every kernel already queued
    on its stream has finished (the U-side launches of ``_msm_queue``)."""
    t = torch.as_tensor(np.asarray(a) if not isinstance(a, torch.Tensor) else a)
    return bn.h2d(t.contiguous(), dev)


def _invalid(valid: torch.Tensor, segs, n_vn: int) -> list:
    if segs is None:
        return [False] * n_vn
    seg_ok = _seg_all(valid.view(1, -1), segs, valid.device).view(-1).tolist()
    return [RangeInvalid(seg_ok) for _ in range(n_vn)]


def _seg_all(flags: torch.Tensor, counts, dev) -> torch.Tensor:
    """[G, k] bool: all(flags[v, run s]) for the consecutive runs of ``counts``."""
    G, nq = flags.shape
    k = len(counts)
    if k == 1:
        return flags.all(dim=1).view(G, 1)
    sid = torch.repeat_interleave(torch.arange(k, device=dev), _h2d(counts, dev), output_size=nq)
    bad = torch.zeros((G, k), dtype=torch.int32, device=dev)
    bad.index_add_(1, sid, (~flags).to(torch.int32))
    return bad == 0


def _seg_products(msq: dict) -> torch.Tensor:
    """Per-(VN, segment) products of the fold partials -> host [G, k, 96]:
    the blocks of every (VN, segment) gathered into one [blocks, G k] image
    (short segments padded with ones), 8-way device levels, then the host."""
    fb, G, blk, sb, nb = msq["fb"], msq["G"], msq["blk"], msq["sb"], msq["nb"]
    k = len(sb)
    dev = fb.device
    maxb = max(nb)
    b = torch.arange(maxb, device=dev).view(maxb, 1, 1)
    base = (torch.arange(G, device=dev).view(1, G, 1) * blk + _h2d(sb, dev).view(1, 1, k))
    idx = torch.where(b < _h2d(nb, dev).view(1, 1, k), base + b, fb.shape[0])
    ext = torch.cat([fb, nt.gt_one(dev)])
    x = ext.index_select(0, idx.reshape(-1)).view(maxb, G * k, 96)
    if dev.type == "cuda":
        while x.shape[0] > 8:
            x = nt._gt_prod_level(x, 8)
    return nt.gt_prod(x.cpu(), chunk=64).view(G, k, 96)  # host: one chain per (VN, segment)


def _seg_c(n_entries: int, n_groups: int, bits: int = 254) -> int:
    """Window of a grouped G2 MSM: entries x windows bucket additions plus a
    per-(group, window, digit) bucket cost of ~36 -- its weight on the device
    and, dominating since the weights are running sums
    (``nt.g2_chunk_weight``), its share of the host-side plan (counts copy,
    nonzero/unique, chunk layout): a 13-bit window over 30 groups measured
    72 ms of planning against 25 ms at 9 bits."""
    return min(range(6, 14), key=lambda c: -(-bits // c) * (n_entries + n_groups * (1 << c) * 36))


def _attribute_hinted(r: RangeProofList, segs: list, redo: list, x: dict) -> dict:
    """Attribution of several failing VNs: the first pays the full
    segment-grouped pass (``_segment_pass``); its failing segments T are then
    the hint for the others, each of which evaluates only T's segments
    (``_segment_hinted``: ~|T|/nseg of the pass) and checks the REST of its
    batch in one equation -- its first-pass totals divided by T's parts (the
    pairing is bilinear on the G2 points it checks, so the rest's equation is
    exactly the batch check of the other segments' proofs with the same
    weights).  A rest that fails, or a hint that explains nothing, falls back
    to the full pass.  -> {vn: [bool] per segment}."""
    out, hint = {}, None
    for v in redo:
        if hint is not None:
            with timers.span("rp.seg.hinted"):
                got = _segment_hinted(r, segs, v, hint, x)
            if got is not None:
                out[v] = got
                continue
        out.update(_segment_pass(r, segs, [v], x))
        bad = [s for s, ok in enumerate(out[v]) if not ok]
        if hint is None and 0 < len(bad) < len(segs):
            hint = bad
    return out


def _segment_hinted(r: RangeProofList, segs: list, v: int, T: list, x: dict):
    """VN ``v``'s per-segment verdicts from the suspect segments ``T`` alone:
    the segment pass over T's proofs (same weights) gives T's per-segment
    equation sides; the rest's sides are the first-pass totals minus T's --
      lhs_rest = lhs_all / prod_T lhs_s,   e_rest = e_all - sum_T e_s,
      D-check: dl_all - sum_T dl_s == dr_all - sum_T dr_s,
      GT membership (when the first-pass combination failed): GGgam_all / prod_T GGgam_s
    with R_all and every R_s, U_q of the rest in G2.  -> [bool] per segment,
    or None when the rest fails or T's segments all pass (no attribution from
    the hint: the caller runs the full pass)."""
    dev = r.V.device
    n, S, l, G = len(r), r.S, r.l, x["G"]
    m, tot = n * S * l, x["tot"]
    if tot["lhs"][v] is None or tot["dl"][v] is None:
        return None
    poff = np.cumsum([0] + list(segs))
    rT = rpl_cat([rpl_range(r, int(poff[s]), int(poff[s + 1])) for s in T])
    pidx = torch.cat([torch.arange(int(poff[s]), int(poff[s + 1])) for s in T])
    iidx = (pidx.view(-1, 1) * (S * l) + torch.arange(S * l).view(1, -1)).reshape(-1)
    pidx, iidx = bn.h2d(pidx, dev), bn.h2d(iidx, dev)
    sel = lambda t, w, idx: t.view(G, -1, w)[v].index_select(0, idx).contiguous()  # noqa: E731
    Tt = bn.h2d(torch.tensor(T), x["u_seg"].device)
    xT = dict(A2=x["A2"].index_select(0, torch.cat([iidx, iidx + m])), rho=sel(x["rho"], 8, iidx),
              ab=sel(x["ab"], 2, iidx), gam=sel(x["gam"], 8, iidx), w=sel(x["w"], 8, pidx),
              Cp=x["Cp"].index_select(0, pidx), z=x["z"].index_select(0, pidx),
              useg=x["useg"][v: v + 1, T], u_seg=x["u_seg"][v: v + 1].index_select(1, Tt),
              PB_base=x["PB_base"], gt_tab=x["gt_tab"], wc=x["wc"], G=1, m_first=[x["m_first"][v]])
    comp = {}
    perT = _segment_pass(rT, [segs[s] for s in T], [0], xT, comp)[0]
    if all(perT):
        return None
    # the rest, from the totals
    inv_lhs = nt.gt_inv(nt.gt_prod(comp["lhs"].view(len(T), 1, 96), chunk=64).view(1, 96))
    lhs_rest = nt.gt_mul(tot["lhs"][v].view(1, 96), inv_lhs)
    e_rest = tot["e"][v: v + 1].cpu()
    for s_ in range(len(T)):
        e_rest = nt.fr_arith(nt.FR_SUB, e_rest, comp["e"][s_: s_ + 1].contiguous())
    eq = bool(nt.gt_eq(lhs_rest, nt.gt_fb_pow(x["gt_tab"], e_rest)).all())
    d1 = nt.g1_sum(torch.cat([tot["dl"][v].view(1, 1, 24), comp["dr"].view(-1, 1, 24)]))
    d2 = nt.g1_sum(torch.cat([tot["dr"][v].view(1, 1, 24), comp["dl"].view(-1, 1, 24)]))
    d_ok = bool(nt.g1_eq(d1, d2)[0])
    m_ok = True
    if not x["m_first"][v]:
        if comp.get("GGgam") is None:
            return None
        gi = nt.gt_inv(nt.gt_prod(comp["GGgam"].view(len(T), 1, 96), chunk=64).view(1, 96))
        m_ok = _gt_in_subgroup(nt.gt_mul(tot["GGgam"][v: v + 1].cpu(), gi))
    rest = [s for s in range(len(segs)) if s not in set(T)]
    u_ok = bool(x["u_seg"][v].cpu()[rest].all()) if rest else True
    g2_ok = tot["r_ok"][v] and all(comp["rok"]) and u_ok
    if not (eq and d_ok and m_ok and g2_ok):
        return None
    out = [True] * len(segs)
    for s_, s in enumerate(T):
        out[s] = perT[s_]
    return out


def _segment_pass(r: RangeProofList, segs: list, redo: list, x: dict, comp: dict | None = None) -> dict:
    """Second, segment-grouped pass for the VNs ``redo`` whose batch failed:
    with the SAME weights, every side of the batch equation per (VN,
    segment) -- R MSM, prod a^rho, sum rho Zv, D-check, GT membership -- in
    one grouped MSM / multi-exponentiation each; the U side's per-segment products come from
    the first pass.  -> {vn: [bool] per segment}; ``comp`` receives the
    per-(VN, segment) sides (host): lhs, e, dl, dr, GGgam (when computed), rok."""
    dev = r.V.device
    n, S, l = len(r), r.S, r.l
    m, nseg, Gf = n * S * l, len(segs), len(redo)
    K = Gf * nseg
    poff = np.cumsum([0] + list(segs))
    pseg = torch.repeat_interleave(torch.arange(nseg, device=dev), _h2d(segs, dev), output_size=n)
    iseg = pseg.repeat_interleave(S * l)
    fi = torch.arange(Gf, device=dev).view(Gf, 1)
    def rows(t, w):
        return torch.cat([t[v * w:(v + 1) * w] for v in redo]) if Gf > 1 else t[redo[0] * w:(redo[0] + 1) * w]

    rho, ab, w = rows(x["rho"], m), rows(x["ab"], m), rows(x["w"], n)
    # every input and every bucket plan (one host sync each) first, then the
    # device passes: a plan's sync then never waits behind another MSM's
    # queued passes (the first pass's schedule)
    # R_(v,s) = sum_{it in s} rho_it Zphi_(p,j) V_it
    it = torch.arange(m, device=dev)
    zi = (it // (S * l)) * l + it % l
    s_r = nt.fr_arith(nt.FR_MUL, rho, r.zphi.index_select(0, zi).contiguous())
    grp = (fi * nseg + iseg.view(1, m)).reshape(-1).to(torch.int32)
    # prod a^rho per (v, s) (32-bit halves over (A, frob^8 A)) and -- only
    # for a VN whose first-pass GT-membership combination failed -- each
    # segment's own combination prod a^gamma (the VN's gammas).  A passing
    # first-pass combination already bounds any non-GT component of the
    # whole batch (error ~2^-38.8), so its segments skip that 40% of the
    # multi-exponentiation
    gam_groups = 2 if any(not x["m_first"][v] for v in redo) else 1
    k = torch.zeros((gam_groups * Gf, 2 * m, 8), dtype=torch.int32, device=dev)
    abv = ab.view(Gf, m, 2)
    k[:Gf, :m, 0] = abv[:, :, 0]
    k[:Gf, m:, 0] = abv[:, :, 1]
    if gam_groups == 2:
        k[Gf:, :m] = rows(x["gam"], m).view(Gf, m, 8)
    k = k.view(-1, 8)
    fi2 = torch.arange(gam_groups * Gf, device=dev).view(gam_groups * Gf, 1)
    grp2 = (fi2 * nseg + iseg.repeat(2).view(1, 2 * m)).reshape(-1).to(torch.int32)
    # D-check per (v, s): sum w c C' - sum w D (groups (v, which, s))
    wc = nt.fr_arith(nt.FR_MUL, w, r.challenge.contiguous())
    dsc = torch.stack([wc.view(Gf, n, 8), w.view(Gf, n, 8)], 1).reshape(-1, 8).contiguous()
    grp3 = ((fi.view(Gf, 1, 1) * 2 + torch.arange(2, device=dev).view(1, 2, 1)) * nseg
            + pseg.view(1, 1, n)).reshape(-1).to(torch.int32)
    dpts = torch.cat([x["Cp"].contiguous(), r.D.contiguous()]).repeat(Gf, 1)
    with timers.span("rp.seg.plans"):
        hR = nt.g2_msm_launch(r.V, s_r, grp, K, c=_seg_c(Gf * m, K))
        mplan = nt.multi_exp_plan(k, grp2, gam_groups * K, W=x["wc"][0], c=x["wc"][1])
        dplan = nt.g1_msm_plan(dsc, grp3, 2 * K)
    with timers.span("rp.seg.passes"):
        S_R = nt.g2_msm_run(r.V, hR)
        mexp = nt.multi_exp_grouped(x["A2"], k, grp2, gam_groups * K, W=x["wc"][0], c=x["wc"][1], plan=mplan)
        dh = nt.g1_msm_launch(dpts, dsc, grp3, 2 * K, bits=256, plan=dplan)
    # sum rho Zv, sum w Zr, sum w z per (v, s): per-proof sums, then per-segment
    offs = torch.from_numpy((np.arange(Gf).reshape(Gf, 1) * n + poff[:-1].reshape(1, nseg)).reshape(-1))
    offs = bn.h2d(torch.cat([offs, torch.tensor([Gf * n])]), dev)
    e = nt.fr_seg_sum(nt.fr_dot_rows(rho, r.zv.repeat(Gf, 1).contiguous(), Gf * n), offs)
    dzr = nt.fr_seg_sum(nt.fr_arith(nt.FR_MUL, w, r.zr.contiguous()), offs)
    dz = nt.fr_seg_sum(nt.fr_arith(nt.FR_MUL, w, x["z"].contiguous()), offs)
    # host: Horner steps, Miller loops of B with each R_(v,s), final exps
    with timers.span("rp.seg.gt_finish"):
        GG = nt.multi_exp_grouped_finish(mexp)                         # [gam_groups * K, 96]
        m_ok = _gt_in_subgroup_each(GG[K:]) if gam_groups == 2 else [True] * K
    if comp is not None and gam_groups == 2:
        comp["GGgam"] = GG[K:].cpu()
    GG = GG[:K]
    with timers.span("rp.seg.r_finish"):
        fR, rok = _msm_r_miller(hR, S_R)
    with timers.span("rp.seg.d_finish"):
        D_all = nt.g1_msm_finish(dh).view(Gf, 2, nseg, 24)
    e, dzr, dz = e.cpu(), dzr.cpu(), dz.cpu()
    useg = torch.stack([x["useg"][v] for v in redo]).view(K, 96)
    useg_ok = x["u_seg"].cpu()[redo].reshape(-1).tolist()
    lhs = nt.gt_mul(nt.final_exp(nt.gt_mul(useg.contiguous(), fR.contiguous())), GG.contiguous())
    eq = nt.gt_eq(lhs, nt.gt_fb_pow(x["gt_tab"], e)).tolist()
    PB = nt.g1_mul(x["PB_base"].repeat(K, 1), torch.stack([dzr, dz], 1).reshape(-1, 8).contiguous()).view(K, 2, 24)
    lhs_d = nt.g1_sum(torch.stack([D_all[:, 0].reshape(K, 24), PB[:, 0], PB[:, 1]]).contiguous())
    d_ok = nt.g1_eq(lhs_d.contiguous(), D_all[:, 1].reshape(K, 24).contiguous()).tolist()
    if comp is not None:
        comp.update(lhs=lhs, e=e, dl=lhs_d, dr=D_all[:, 1].reshape(K, 24), rok=rok)
    out = {}
    for f, v in enumerate(redo):
        out[v] = [bool(eq[f * nseg + s_]) and bool(d_ok[f * nseg + s_]) and bool(useg_ok[f * nseg + s_])
                  and bool(rok[f * nseg + s_]) and m_ok[f * nseg + s_] for s_ in range(nseg)]
    return out


def _msm_r_miller(hR, S_dev) -> torch.Tensor:
    """Host tail of the R side: Horner over the window sums (one core per VN
    beats one GPU lane at this serial chain) and ML(B, R_v) -> ([G, 96] host,
    [R_v in G2] per VN)."""
    R = nt.g2_msm_finish(S_dev.cpu(), hR)
    B = nt.g1_to_affine(bn.g1_jac_tensor([O.G1_GEN], "cpu")).repeat(R.shape[0], 1)
    f = nt.miller_loop(B, R)
    inf = ~R.bool().any(dim=1)                                         # R = O: e(B, O) = 1
    if bool(inf.any()):
        f[inf] = nt.gt_one("cpu")
    return f, [bool(x) for x in nt.g2_subgroup(R).tolist()]


def fold_k(n_items: int, slots: int = 2048) -> int:
    """Items per lane of the multi-Miller accumulation: a workgroup's time is
    ~ (12 + 13 K) Fp2 products per loop step (one shared squaring, K sparse
    line products) and up to ``slots`` workgroups (2 waves on each of the
    1024 SIMDs) run per round -> minimise rounds x (12 + 13 K)."""
    best, best_k = None, 1
    for k in (1, 2, 4, 8):
        wgs = -(-n_items // (64 * k))
        cost = -(-wgs // slots) * (12 + 13 * k)
        if best is None or cost < best:
            best, best_k = cost, k
    return best_k


# U-side items up to which the accumulation runs three lanes per item (one
# item per lane would leave most SIMDs idle; 43008 items = 2048 coop waves)
_COOP_MAX_ITEMS = 43008

_aux: dict = {}
_val: dict = {}


def _val_stream(device):
    key = str(device)
    if key not in _val:
        _val[key] = torch.cuda.Stream(device, priority=streams.priority(VAL_PRIORITY))
    return _val[key]


AUX_PRIORITY = -1  # A/B constants (tools/ab_patch.py --aux-priority / --val-priority)
VAL_PRIORITY = 0


def _aux_stream(device):
    key = str(device)
    if key not in _aux:
        # plans: short kernels overtake the pairing side
        _aux[key] = torch.cuda.Stream(device, priority=streams.priority(AUX_PRIORITY))
    return _aux[key]


def rpl_cat(lists: list) -> RangeProofList:
    """Concatenate proof lists sharing (u, l, S) into one batch (columnar)."""
    r0 = lists[0]
    if len(lists) == 1:
        return r0
    assert all((r.u, r.l, r.S) == (r0.u, r0.l, r0.S) for r in lists)
    # every field of every list in ONE batched-copy launch (torch.cat ran each
    # field as its own ~50-workgroup kernel: ~10 ms per inbox on the trace)
    fields = ("challenge", "zr", "D", "zphi", "zv", "V", "A")
    have = [f for f in fields if getattr(r0, f) is not None]
    outs = nt.cat_rows([[r.commit.K for r in lists], [r.commit.C for r in lists]]
                       + [[getattr(r, f) for r in lists] for f in have])
    got = dict(zip(have, outs[2:]))
    return RangeProofList(r0.u, r0.l, r0.S, [o for r in lists for o in r.offset], [c for r in lists for c in r.cols],
                          CipherVector(outs[0], outs[1]), *[got.get(f) for f in fields])


def rpl_range(r: RangeProofList, a: int, b: int) -> RangeProofList:
    """Proofs a..b-1 of a list (views)."""
    l, S = r.l, r.S
    sl = lambda t, w: None if t is None else t[a * w: b * w]  # noqa: E731
    return RangeProofList(r.u, l, S, r.offset[a:b], r.cols[a:b], r.commit[a:b], sl(r.challenge, 1), sl(r.zr, 1),
                          sl(r.D, 1), sl(r.zphi, l), sl(r.zv, S * l), sl(r.V, S * l), sl(r.A, S * l))


def _slice(r: RangeProofList, k: int) -> RangeProofList:
    l, S = r.l, r.S
    return RangeProofList(r.u, l, S, r.offset[:k], r.cols[:k], r.commit[:k], r.challenge[:k], r.zr[:k], r.D[:k],
                          r.zphi[: k * l], r.zv[: k * S * l], r.V[: k * S * l], r.A[: k * S * l])


def verify_range_proof_single_reference(rpl: RangeProofList, p: int, sigmat: SigMaterial, P_point) -> bool:
    """Unbatched, equation-by-equation check of proof p exactly as
    range_proof.go:504-565 (3 pairings per (i, j)); used to cross-check the
    batched verifier in tests."""
    device = rpl.commit.device
    n, l, S, u = len(rpl), rpl.l, rpl.S, rpl.u
    c = bn.scalars_from_tensor(rpl.challenge[p: p + 1])[0]
    zr = bn.scalars_from_tensor(rpl.zr[p: p + 1])[0]
    zphi = bn.scalars_from_tensor(rpl.zphi[p * l:(p + 1) * l])
    zv = bn.scalars_from_tensor(rpl.zv[p * S * l:(p + 1) * S * l])
    Cpt = bn.g1_points_from_jac(rpl.commit.C[p: p + 1])[0]
    Cpt = O.g1_add(Cpt, O.g1_mul_signed(rpl.offset[p], O.G1_GEN)) if rpl.offset[p] else Cpt
    D = bn.g1_points_from_jac(rpl.D[p: p + 1])[0]
    Dp = O.g1_add(O.g1_mul(c, Cpt), O.g1_mul(zr, P_point))
    for j in range(l):
        Dp = O.g1_add(Dp, O.g1_mul(zphi[j] * pow(u, j, O.R), O.G1_GEN))
    if Dp != D:
        return False
    V = rpl.V[p * S * l:(p + 1) * S * l]
    A = rpl.A[p * S * l:(p + 1) * S * l]
    Pa, Qa = [], []
    for i in range(S):
        y = sigmat.y_pts[i * sigmat.n_cols + rpl.cols[p]]
        for j in range(l):
            Pa += [O.g1_mul(c, y), O.g1_mul((-zphi[j]) % O.R, O.G1_GEN), O.g1_mul(zv[i * l + j], O.G1_GEN)]
            Qa += [i * l + j, i * l + j, None]
    Vp = bn.g2_points_from_aff(V)
    Qpts = [Vp[q] if q is not None else O.G2_GEN for q in Qa]
    e = nt.pairing(bn.g1_aff_tensor(Pa, device), bn.g2_aff_tensor(Qpts, device))
    e3 = e.view(-1, 3, 96)
    prod = nt.gt_mul(nt.gt_mul(e3[:, 0].contiguous(), e3[:, 1].contiguous()), e3[:, 2].contiguous())
    return bool(nt.gt_eq(prod, A.contiguous()).all())
