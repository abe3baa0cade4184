"""K14 exact int64 moments and the batched many-DP encoder.

The kernel (csrc/kernels/dx_moments.hip) is checked against a plain-Python
int64 reference of the same sums (reference encoders: lib/encoding/sum.go,
variance.go:21-24, cosim.go:26-34, linear_regression_dims.go:48-89,
model_evaluation.go:33-37); the batched encoder against the per-DP encoder
(clear values and decrypted ciphertexts)."""
import pytest
import torch

from drynx_amd import native as nt
from drynx_amd.crypto import elgamal as eg
from drynx_amd.crypto import oracle as O
from drynx_amd.ops import encoding as enc
from drynx_amd.protocols import data_collection as dcp
from drynx_amd.services.api import DrynxClient
from drynx_amd.services.local import local_cluster, make_survey

M64 = 1 << 64


def _wrap(v: int) -> int:
    v %= M64
    return v - M64 if v >= 1 << 63 else v


def _ref_moments(Z, counts, pairs):
    C = Z.shape[1]
    rows = Z.tolist()
    out, s = [], 0
    for c in counts:
        blk = rows[s: s + c]
        s += c
        out.append([_wrap(sum((r[a] if a < C else 1) * (r[b] if b < C else 1) for r in blk)) for a, b in pairs])
    return out


@pytest.mark.parametrize("C,counts,lo,hi", [
    (1, [5], -10, 10),
    (3, [0, 1, 130, 64, 0, 7], -1000, 1000),
    (9, [700, 1, 1, 3], 0, 4),
    (2, [40], -(1 << 40), 1 << 40),  # products wrap mod 2^64 like Go int64
])
def test_int_moments_cpu_matches_reference(C, counts, lo, hi):
    g = torch.Generator().manual_seed(C * 7 + len(counts))
    Z = torch.randint(lo, hi, (sum(counts), C), generator=g, dtype=torch.int64)
    pairs = [(a, b) for a in range(C + 1) for b in range(a, C + 1)]
    out = nt.int_moments(Z, counts, pairs)
    assert out.tolist() == _ref_moments(Z, counts, pairs)


def test_int_moments_rejects_bad_shapes():
    Z = torch.zeros((4, 2), dtype=torch.int64)
    with pytest.raises(ValueError):
        nt.int_moments(Z, [4], [(0, 3)])  # column 3 > C
    with pytest.raises(ValueError):
        nt.int_moments(Z, [3], [(0, 1)])  # segments do not cover the rows
    with pytest.raises(ValueError):
        nt.int_moments(torch.zeros((1, 65), dtype=torch.int64), [1], [(0, 0)])


@pytest.mark.parametrize("op,d", [("sum", 1), ("mean", 1), ("variance", 1), ("cosim", 1), ("lin_reg", 3),
                                  ("MLeval", 1)])
def test_moment_encoders_match_python(op, d):
    g = torch.Generator().manual_seed(3)
    n_in = {"cosim": 2, "MLeval": 2, "lin_reg": d + 1}.get(op, 1)
    cols = [torch.randint(-50, 50, (37,), generator=g, dtype=torch.int64) for _ in range(n_in)]
    Z = torch.stack(cols, 1)
    got = enc.batch_values(op, Z, [37])[0].tolist()
    c = [x.tolist() for x in cols]
    S = lambda v: sum(v)  # noqa: E731
    if op == "sum":
        exp = [S(c[0])]
    elif op == "mean":
        exp = [S(c[0]), 37]
    elif op == "variance":
        exp = [S(c[0]), 37, S(x * x for x in c[0])]
    elif op == "cosim":
        a, b = c
        exp = [S(a), S(b), S(x * x for x in a), S(x * x for x in b), S(x * y for x, y in zip(a, b))]
    elif op == "MLeval":
        y, p = c
        exp = [37, S(y), S(x * x for x in y), S((q - x) ** 2 for x, q in zip(y, p))]
    else:  # linear_regression_dims.go:48-89 output order
        X, y = c[:-1], c[-1]
        exp = [37] + [S(x) for x in X]
        exp += [S(u * v for u, v in zip(X[j], X[k])) for j in range(d) for k in range(j, d)]
        exp += [S(y)] + [S(u * v for u, v in zip(X[j], y)) for j in range(d)]
    assert got == exp


@pytest.fixture(scope="module")
def env(tmp_path_factory):
    cl, node = local_cluster(3, 6, 1, device="cpu", workdir=str(tmp_path_factory.mktemp("db")))
    yield cl, node, DrynxClient(node)
    node.close(remove=True)


@pytest.mark.parametrize("op", sorted(enc.BATCH_OPS))
@pytest.mark.parametrize("proofs", [0, 1])
def test_batched_encoder_matches_per_dp(env, op, proofs):
    cl, node, client = env
    sq = make_survey(client, cl, op, query_min=0, query_max=5, rows=9, d=2, group_by=(2,), proofs=proofs,
                     ranges=[16, 16] if proofs else None, deterministic_sigs=True)
    dps = list(cl.dps)
    batch = dcp.dp_encode_batch(node, sq, dps)
    secret = sum(cn.keypair.secret for cn in cl.cns) % O.R
    bits = op in enc.BIT_OPS
    for dp in dps:
        single = dcp.dp_encode(node, sq, dp)
        b = batch[dp.id]
        assert b["clear"] == single["clear"] and b["n_groups"] == single["n_groups"] == 2
        assert len(b["cv"]) == len(single["cv"])
        if bits and not proofs:
            assert (eg.decrypt_check_zero(secret, b["cv"]).tolist()
                    == eg.decrypt_check_zero(secret, single["cv"]).tolist())
        else:
            assert eg.decrypt_ints(secret, b["cv"]) == [v for grp in b["clear"] for v in grp]
        if proofs:
            assert len(b["proofs"]) == 2
            for pb, ps in zip(b["proofs"], single["proofs"]):
                assert pb.values == ps.values and pb.u == ps.u and pb.l == ps.l and pb.sig_col == ps.sig_col
                # the proof's (value, r) opens the ciphertext it proves
                cv2, _ = eg.encrypt_ints(eg.pk_table(sq.RosterServers.aggregate()), pb.values, pb.r)
                assert torch.equal(nt.g1_to_affine(cv2.K), nt.g1_to_affine(pb.cv.K))
                assert torch.equal(nt.g1_to_affine(cv2.C), nt.g1_to_affine(pb.cv.C))


def test_batched_encoder_cutting_factor(env):
    cl, node, client = env
    sq = make_survey(client, cl, "sum", query_min=0, query_max=5, rows=4, cutting_factor=2, d=1)
    sq.Query.Operation.NbrOutput = 2
    batch = dcp.dp_encode_batch(node, sq, list(cl.dps))
    secret = sum(cn.keypair.secret for cn in cl.cns) % O.R
    for dp in cl.dps:
        b = batch[dp.id]
        assert len(b["cv"]) == 2  # the one output replicated CuttingFactor times (same ciphertext)
        assert torch.equal(b["cv"].K[0], b["cv"].K[1])
        assert eg.decrypt_ints(secret, b["cv"]) == b["clear"][0] * 2


@pytest.mark.parametrize("proofs", [0, 1])
def test_batched_lr_encoder_matches_per_dp(env, proofs):
    """Logistic regression through the batched encoder (per-DP fused encoder,
    one encryption launch for all DPs) == the per-DP path."""
    from drynx_amd.query import LogisticRegressionParameters

    cl, node, client = env
    d = 3
    lp = LogisticRegressionParameters(NbrRecords=24, NbrFeatures=d, Means=[0.5] * d, StandardDeviations=[1.1] * d,
                                      Lambda=1.0, Step=0.1, MaxIterations=5, InitialWeights=[0.1] * (d + 1), K=2,
                                      PrecisionApproxCoefficients=100.0)
    sq = make_survey(client, cl, "logistic regression", proofs=proofs, ranges=[16, 8, 1 << 31] if proofs else None,
                     lr_params=lp, deterministic_sigs=True)
    dps = list(cl.dps)
    batch = dcp.dp_encode_batch(node, sq, dps)
    secret = sum(cn.keypair.secret for cn in cl.cns) % O.R
    for dp in dps:
        single = dcp.dp_encode(node, sq, dp)
        b = batch[dp.id]
        assert b["clear"] == single["clear"]
        assert eg.decrypt_ints(secret, b["cv"]) == [v for grp in b["clear"] for v in grp]
        if proofs:
            for pb, ps in zip(b["proofs"], single["proofs"]):
                assert pb.values == ps.values and pb.offset == ps.offset and pb.u == ps.u and pb.l == ps.l
