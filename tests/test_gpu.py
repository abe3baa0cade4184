"""GPU (gfx950) kernels vs the host path / oracle.  Run with -m gpu on an MI355X."""
import random

import pytest
import torch

from drynx_amd import native as nt
from drynx_amd.crypto import bn254 as bn
from drynx_amd.crypto import oracle as O

pytestmark = pytest.mark.gpu
RNG = random.Random(11)


def _both(fn, *cpu_args):
    """Run fn on CPU and on GPU copies of the args; return (cpu, gpu->cpu)."""
    dev = torch.device("cuda", 0)
    c = fn(*cpu_args)
    g = fn(*[a.to(dev) if isinstance(a, torch.Tensor) else a for a in cpu_args])
    torch.cuda.synchronize()
    return c, (g.cpu() if isinstance(g, torch.Tensor) else g)


def test_native_loaded_on_gpu(gpu_device):
    assert nt.lib().dx_version() == 1
    assert nt.loaded_path().endswith("libdrynx_native.so")


def test_g1_ops_gpu_match_cpu(gpu_device):
    ks = bn.scalars_tensor([RNG.randrange(O.R) for _ in range(300)] + [0, 1, O.R - 1])
    c, g = _both(lambda k: nt.g1_fb_mul(bn.base_table(k.device), k), ks)
    assert torch.equal(nt.g1_to_affine(c), nt.g1_to_affine(g))
    J = bn.g1_jac_tensor([O.g1_mul(5, O.G1_GEN)])
    c, g = _both(lambda j, k: nt.g1_to_affine(nt.g1_mul(j, k)), J, ks)
    assert torch.equal(c, g)
    x = bn.g1_jac_tensor([O.g1_mul(i + 1, O.G1_GEN) for i in range(40)]).view(8, 5, 24)
    c, g = _both(lambda t: nt.g1_to_affine(nt.g1_sum(t)), x)
    assert torch.equal(c, g)


def test_fr_and_codecs_gpu(gpu_device):
    a = bn.scalars_tensor([RNG.randrange(O.R) for _ in range(100)])
    b = bn.scalars_tensor([RNG.randrange(O.R) for _ in range(100)])
    for op in (nt.FR_ADD, nt.FR_SUB, nt.FR_MUL):
        c, g = _both(lambda x, y: nt.fr_arith(op, x, y), a, b)
        assert torch.equal(c, g)
    pts = [O.g1_mul(RNG.randrange(O.R), O.G1_GEN) for _ in range(10)]
    t = bn.g1_aff_tensor(pts, gpu_device)
    assert bytes(bn.g1_aff_to_bytes(t).tobytes()) == b"".join(O.g1_to_bytes(p) for p in pts)


def test_pairing_gpu_matches_oracle(gpu_device):
    P = [O.g1_mul(RNG.randrange(1, O.R), O.G1_GEN) for _ in range(64)]
    Q = [O.g2_mul(RNG.randrange(1, O.R), O.G2_GEN) for _ in range(2)] * 32
    Pt, Qt = bn.g1_aff_tensor(P), bn.g2_aff_tensor(Q)
    c, g = _both(nt.pairing, Pt, Qt)
    assert torch.equal(c, g)
    assert bn.gt_from_tensor(g[:1])[0] == O.pairing(P[0], Q[0])
    c, g = _both(lambda p, q: nt.final_exp(nt.miller_loop(p, q)), Pt[:8], Qt[:8])
    assert torch.equal(c, g)


def test_g2_and_gt_gpu(gpu_device):
    ks = bn.scalars_tensor([RNG.randrange(O.R) for _ in range(64)])
    c, g = _both(lambda k: nt.g2_fb_mul(bn.base2_table(k.device), k), ks)
    assert torch.equal(c, g)
    c, g = _both(lambda k: nt.g2_mul(bn.g2_generator_aff(k.device), k), ks)
    assert torch.equal(c, g)
    e = nt.pairing(bn.g1_generator_aff(), bn.g2_generator_aff())
    c, g = _both(lambda t, k: nt.gt_pow(t, k), e, ks[:16].contiguous())
    assert torch.equal(c, g)


def test_elgamal_and_bsgs_gpu(gpu_device):
    from drynx_amd.crypto import elgamal as eg

    kp = eg.KeyPair.generate()
    pk = eg.pk_table(kp.public, gpu_device)
    vals = [RNG.randrange(-10**6, 10**6) for _ in range(500)]
    cv, _ = eg.encrypt_ints(pk, vals)
    assert eg.decryption_table(10**6, gpu_device).decrypt(kp.secret, cv).cpu().tolist() == vals
    big = [10**9 + 7, -(10**9) + 3]
    cv2, _ = eg.encrypt_ints(pk, big)
    assert eg.decrypt_auto(kp.secret, cv2, 10000).cpu().tolist() == big


def test_lr_moments_mfma_matches_fp64(gpu_device):
    for N, D in [(1000, 45), (4099, 9), (123, 48)]:
        X = torch.randn(N, D, dtype=torch.float64, device=gpu_device)
        w = torch.randn(N, dtype=torch.float64, device=gpu_device)
        ref = (X * w[:, None]).T @ X
        got = nt.lr_moments(X, w)
        assert torch.allclose(got, ref, rtol=1e-10, atol=1e-9), (got - ref).abs().max()


def test_lr_encode_fused_matches_torch(gpu_device):
    """Fused standardise+augment+level1+level2 kernel vs the plain torch path."""
    from drynx_amd.models import logistic_regression as lr

    for N, d in [(5000, 44), (1001, 8), (77, 46)]:
        X = torch.rand(N, d, dtype=torch.float64, device=gpu_device) * 4
        y = torch.randint(0, 2, (N,), device=gpu_device)
        m, s = lr.compute_means_sds(X)
        Xa = lr.augment((X - m) / s)
        yf = y.to(torch.float64)
        ref1 = Xa.T @ (2 * yf - 1)
        ref2 = -(Xa.T @ Xa)
        g1, g2 = nt.lr_encode(X, y, m, s, 0.0, -1.0)
        assert torch.allclose(g1, ref1, rtol=1e-10, atol=1e-8), (g1 - ref1).abs().max()
        assert torch.allclose(g2, ref2, rtol=1e-10, atol=1e-8), (g2 - ref2).abs().max()


def test_lr_encode_many_matches_single(gpu_device):
    """Several DPs through one encoder batch (one reduction launch) == each DP
    alone, bit for bit, and == the plain torch fp64 reference; the rounded
    coefficient vectors of the batch == encode_coefficients_int per DP."""
    from drynx_amd.models import logistic_regression as lr
    from drynx_amd.query import LogisticRegressionParameters

    d = 44
    Xs = [torch.rand(n, d, dtype=torch.float64, device=gpu_device) * 4 for n in (3000, 3000, 517, 80001)]
    ys = [torch.randint(0, 2, (X.shape[0],), device=gpu_device) for X in Xs]
    m, s = [2.0] * d, [1.15] * d
    tot = nt.lr_encode_many(Xs, ys, m, s, 0.0, -1.0)
    D = d + 1
    mt = torch.tensor(m, dtype=torch.float64, device=gpu_device)
    st = torch.tensor(s, dtype=torch.float64, device=gpu_device)
    for i, (X, y) in enumerate(zip(Xs, ys)):
        g1, g2 = nt.lr_encode(X, y, mt, st, 0.0, -1.0)
        assert torch.equal(tot[i, D, :D], g1) and torch.equal(tot[i, :D, :D], g2)
        Xa = lr.augment((X - mt) / st)
        ref1 = Xa.T @ (2 * y.to(torch.float64) - 1)
        assert torch.allclose(g1, ref1, rtol=1e-10, atol=1e-8), (g1 - ref1).abs().max()
        assert torch.allclose(g2, -(Xa.T @ Xa), rtol=1e-10, atol=1e-8)
    lp = LogisticRegressionParameters(NbrRecords=1, NbrFeatures=d, Means=m, StandardDeviations=s, Lambda=1.0,
                                      Step=0.1, MaxIterations=5, InitialWeights=[0.1] * D, K=2,
                                      PrecisionApproxCoefficients=100.0)
    many = lr.encode_coefficients_int_many(Xs, ys, lp)
    for i, (X, y) in enumerate(zip(Xs, ys)):
        assert torch.equal(many[i], lr.encode_coefficients_int(X, y, lp))


def test_range_proofs_gpu(gpu_device):
    from drynx_amd.crypto import elgamal as eg
    from drynx_amd.ops.encoding import CreateProofBatch
    from drynx_amd.proofs import range_proof as rp

    S, u, l = 3, 16, 4
    sigs = [[rp.init_range_proof_signature(u, device=gpu_device) for _ in range(4)] for _ in range(S)]
    sm = rp.SigMaterial(sigs, gpu_device)
    P = eg.aggregate_keys([eg.KeyPair.generate().public for _ in range(S)])
    vals = [0, 1, 65535, 1234]
    cv, r = eg.encrypt_ints(eg.pk_table(P, gpu_device), vals)
    rpl = rp.create_range_proofs(CreateProofBatch(vals, r, cv, [u] * 4, [l] * 4, [0, 1, 2, 3], [0] * 4), sm, P,
                                 gpu_device)[0]
    assert rp.verify_range_proof_list(rpl, sm, P, 1.0, gpu_device)
    assert rp.verify_range_proof_single_reference(rpl.to("cpu"), 2, rp.SigMaterial(sigs, "cpu"), P)
    rpl.zv[3, 0] ^= 1
    assert not rp.verify_range_proof_list(rpl, sm, P, 1.0, gpu_device)


def test_survey_end_to_end_gpu(gpu_device, tmp_path):
    from drynx_amd.services.api import DrynxClient
    from drynx_amd.services.local import local_cluster, make_survey

    cl, node = local_cluster(3, 4, 2, device=gpu_device, workdir=str(tmp_path))
    client = DrynxClient(node, device=gpu_device)
    sq = make_survey(client, cl, "variance", query_min=0, query_max=50, rows=100, proofs=1, ranges=[16, 5],
                     sig_device=gpu_device)
    _, vals, res = client.send_survey_query(sq)
    tot = [sum(v[0][i] for v in res.clear_dp.values()) for i in range(3)]
    m = tot[0] / tot[1]
    assert abs(vals[0][0] - (tot[2] / tot[1] - m * m)) < 1e-9
    assert set(res.block.data_block().Proofs.values()) == {1}
    node.close(remove=True)


def test_field_mul_edge_cases_gpu(gpu_device):
    """Device Montgomery product (product-scanning asm path) vs the host CIOS
    path on edge operands (0, 1, r-1, 2^k, values near 2^254)."""
    edge = [0, 1, 2, O.R - 1, O.R - 2, (1 << 253) % O.R, (1 << 128) + 1, 0xFFFFFFFF, (O.R - 1) // 2]
    vals = edge + [RNG.randrange(O.R) for _ in range(400)]
    a = bn.scalars_tensor([x for x in vals for _ in vals[:9]])
    b = bn.scalars_tensor([y for _ in vals for y in vals[:9]])
    for op in (nt.FR_MUL, nt.FR_INV):
        c, g = _both(lambda x, y: nt.fr_arith(op, x, y if op == nt.FR_MUL else None), a, b)
        assert torch.equal(c, g)
    got = bn.scalars_from_tensor(_both(lambda x, y: nt.fr_arith(nt.FR_MUL, x, y), a, b)[1])
    ai, bi = bn.scalars_from_tensor(a), bn.scalars_from_tensor(b)
    assert got == [(x * y) % O.R for x, y in zip(ai, bi)]


def test_shuffle_proof_gpu(gpu_device):
    """DRO shuffle proof on the device (N = 2000): prove, verify, reject a tampered output."""
    from drynx_amd.crypto import elgamal as eg
    from drynx_amd.proofs import aggregation_shuffle as ags
    from drynx_amd.proofs import shuffle as sh

    kp = eg.KeyPair.generate()
    pk = eg.pk_table(kp.public, gpu_device)
    X, _ = eg.encrypt_ints(pk, [RNG.randrange(-50, 50) for _ in range(2000)])
    Y, perm, rho = ags.shuffle_sequence(X, kp.public)
    pr = sh.prove(X, Y, perm, rho, kp.public)
    assert sh.verify(pr, kp.public)
    cpu = sh.ShuffleProof.from_bytes(pr.to_bytes(), "cpu")
    assert sh.verify(cpu, kp.public)
    Y.C[5] = Y.C[6]
    assert not sh.verify(sh.prove(X, Y, perm, rho, kp.public), kp.public)


@pytest.mark.parametrize("op", ["sum", "mean", "variance", "cosim", "frequencyCount", "lin_reg", "MLeval",
                                "min", "max", "bool_OR", "bool_AND", "union", "inter", "logistic regression"])
def test_every_operation_on_gpu(gpu_device, tmp_path, op):
    """Every operation end to end with every party on the GPU (encoders, HIP
    aggregation/key switching/decryption), checked against the clear sum of the
    DPs' answers."""
    from drynx_amd.ops import encoding as enc
    from drynx_amd.query import LogisticRegressionParameters
    from drynx_amd.services.api import DrynxClient
    from drynx_amd.services.local import local_cluster, make_survey

    cl, node = local_cluster(2, 3, 1, device=gpu_device, workdir=str(tmp_path))
    client = DrynxClient(node, device=gpu_device)
    lp = None
    if op == "logistic regression":
        lp = LogisticRegressionParameters(NbrRecords=30, NbrFeatures=3, Means=[0.0] * 3, StandardDeviations=[1.0] * 3,
                                          Lambda=1.0, Step=0.1, MaxIterations=5, InitialWeights=[0.1] * 4, K=2,
                                          PrecisionApproxCoefficients=1e2)
    bool_ops = ("min", "max", "bool_OR", "bool_AND", "union", "inter")
    rows = [[2, 3, 5], [1, 5, 6], [3, 4, 5]]  # bool ops read the DP's first value == 1
    if op in bool_ops:
        node.dp_data = {dp.id: [torch.tensor(rows[i], dtype=torch.int64, device=gpu_device)]
                        for i, dp in enumerate(cl.dps)}
    sq = make_survey(client, cl, op, query_min=0, query_max=6, rows=10 if op not in bool_ops else 3, d=2,
                     lr_params=lp)
    _, vals, res = client.send_survey_query(sq)
    if op in bool_ops:
        sets = [set(r) for r in rows]
        exp = {"min": [1.0], "max": [6.0], "bool_OR": [1.0], "bool_AND": [0.0],
               "union": [float(any(i in s for s in sets)) for i in range(7)],
               "inter": [float(all(i in s for s in sets)) for i in range(7)]}[op]
        assert vals[0] == exp
    elif op == "logistic regression":
        # the weights are the clear-text gradient descent on the clear aggregate
        # of the DPs' coefficient vectors (nothing lost in encryption/decoding)
        from drynx_amd.models.logistic_regression import decode_logistic_regression_values

        n = len(next(iter(res.clear_dp.values()))[0])
        tot = [sum(v[0][i] for v in res.clear_dp.values()) for i in range(n)]
        exp = decode_logistic_regression_values(tot, lp)
        assert len(vals[0]) == 4
        assert vals[0] == pytest.approx(list(exp), rel=1e-9, abs=1e-12)
    else:
        n = sq.Query.Operation.NbrOutput
        tot = [sum(v[0][i] for v in res.clear_dp.values()) for i in range(n)]
        exp = enc.decode_values(op, tot, sq.Query.Operation)
        assert vals[0] == pytest.approx(exp, rel=1e-9, abs=1e-9)
    node.close(remove=True)


def test_two_phase_fold_matches_oracle(gpu_device, variant="inl"):
    """Line image + K-item multi-Miller accumulation == product of the
    oracle's pairings (after one final exponentiation), for every K."""
    m = 67  # a ragged last workgroup for every K
    ks = [RNG.randrange(1, O.R) for _ in range(m)]
    kq = [RNG.randrange(1, O.R) for _ in range(m)]
    P = nt.g1_to_affine(nt.g1_fb_mul(bn.base_table(gpu_device), bn.scalars_tensor(ks, gpu_device)))
    V = nt.g2_fb_mul(bn.base2_table(gpu_device), bn.scalars_tensor(kq, gpu_device))
    P[5] = 0  # a point at infinity contributes 1
    # e(a B, b B2) = gT^(a b): the oracle's product of the pairings
    gT = O.pairing(O.G1_GEN, O.G2_GEN)
    expo = sum(a * b for i, (a, b) in enumerate(zip(ks, kq)) if i != 5) % O.R
    want = gT ** expo
    lines = nt.rp_fold_lines(P, V, variant)
    for K in (1, 2, 4, 8):
        fb = nt.rp_fold_accum(lines, m, K, variant)
        got = nt.final_exp(nt._finish_prod_on_host(fb))
        assert bn.gt_from_tensor(got)[0] == want, K


def test_fb4_combs_match_oracle(gpu_device):
    ks = [RNG.randrange(O.R) for _ in range(40)] + [0, 1, O.R - 1]
    k = bn.scalars_tensor(ks, gpu_device)
    Q = O.g2_mul(RNG.randrange(1, O.R), O.G2_GEN)
    tab = nt.g2_fb4_table(bn.g2_aff_tensor([Q], gpu_device))
    got = bn.g2_points_from_aff(nt.g2_fb4_mul(tab, k).cpu())
    assert got == [O.g2_mul(x, Q) for x in ks]
    e = nt.pairing(bn.g1_generator_aff(gpu_device), bn.g2_aff_tensor([Q], gpu_device))
    gt_tab = nt.gt_fb4_table(e)
    g = bn.gt_from_tensor(nt.gt_fb4_pow(gt_tab, k).cpu())
    e0 = bn.gt_from_tensor(e.cpu())[0]
    assert g[:3] == [e0 ** x for x in ks[:3]]
    assert torch.equal(nt.gt_fb4_pow(gt_tab, k), nt.gt_pow(e.expand(len(ks), 96).contiguous(), k))


@pytest.mark.parametrize("bits", ["8", "7", "6", "4", "0"])
def test_range_prover_layouts_gpu(gpu_device, bits, monkeypatch):
    """Every prover path on the GPU with random per-CN, per-column keys:
    8-bit combs, the HBM-sized 4-bit combs, and the table-free path
    (variable-base G2 + one pairing per item)."""
    from drynx_amd.crypto import elgamal as eg
    from drynx_amd.ops.encoding import CreateProofBatch
    from drynx_amd.proofs import range_proof as rp

    monkeypatch.setenv("DRYNX_PROVER_TABLE_BITS", bits)
    S, u, l, ncol = 3, 16, 4, 5
    sigs = [rp.init_range_proof_signatures([u] * ncol, gpu_device) for _ in range(S)]
    sm = rp.SigMaterial(sigs, gpu_device)
    assert sm.table_mode(gpu_device) == int(bits)
    P = eg.aggregate_keys([eg.KeyPair.generate().public for _ in range(S)])
    vals = [0, 1, 65535, 1234, 999]
    cv, r = eg.encrypt_ints(eg.pk_table(P, gpu_device), vals)
    rpl = rp.create_range_proofs(CreateProofBatch(vals, r, cv, [u] * 5, [l] * 5, list(range(5)), [0] * 5), sm, P,
                                 gpu_device)[0]
    assert rp.verify_range_proof_list(rpl, sm, P, 1.0, gpu_device)
    cpu_sm = rp.SigMaterial(sigs, "cpu")
    assert all(rp.verify_range_proof_single_reference(rpl.to("cpu"), p, cpu_sm, P) for p in (0, 3))
    rpl.A[7, 5] ^= 1
    assert not rp.verify_range_proof_list(rpl, sm, P, 1.0, gpu_device)


def test_fold_points_match_g1_ops(gpu_device, variant="inl"):
    """Fused gather + difference + 64-bit multiplication + affine == the same
    through the separate G1 launches (including Y = infinity rows)."""
    S, L, npj = 3, 4, 5
    ZB = nt.g1_fb_mul(bn.base_table(gpu_device), bn.random_scalars(npj * L, gpu_device))
    Y = nt.g1_fb_mul(bn.base_table(gpu_device), bn.random_scalars(npj * S, gpu_device))
    Y[2] = bn.g1_infinity_jac(1, gpu_device)[0]
    rho = bn.random_scalars(npj * S * L, gpu_device)
    rho[:, 2:] = 0
    got = nt.rp_fold_points(ZB, Y, rho, S, L, variant)
    zb = ZB.view(npj, 1, L, 24).expand(npj, S, L, 24).reshape(-1, 24).contiguous()
    yy = Y.view(npj, S, 1, 24).expand(npj, S, L, 24).reshape(-1, 24).contiguous()
    want = nt.g1_to_affine(nt.g1_mul(nt.g1_add(zb, yy, subtract=True), rho))
    assert torch.equal(got, want)


def test_int_moments_gpu_matches_host(gpu_device):
    """K14 on gfx950 vs the host path: one 1e5-record DP split over many
    workgroups, thousands of one-record DPs, empty DPs, and the widest pair
    list (64 columns + the constant -> 2145 pairs, L = 1, 9 units per thread)."""
    g = torch.Generator().manual_seed(5)
    for C, counts, lo, hi in ((1, [100_000, 3, 0, 77], -(1 << 20), 1 << 20),
                              (9, [1] * 6000 + [0, 64, 65, 129], 0, 4),
                              (64, [1000, 1, 333], -(1 << 40), 1 << 40)):
        Z = torch.randint(lo, hi, (sum(counts), C), generator=g, dtype=torch.int64)
        pairs = [(a, b) for a in range(C + 1) for b in range(a, C + 1)]
        c, gg = _both(lambda z: nt.int_moments(z, counts, pairs), Z)
        assert torch.equal(c, gg), C


def test_batched_dp_encoding_gpu(gpu_device, tmp_path):
    """All DPs of a rank encoded as one batch on the GPU == the per-DP encoder."""
    from drynx_amd.crypto import elgamal as eg
    from drynx_amd.protocols import data_collection as dcp
    from drynx_amd.services.api import DrynxClient
    from drynx_amd.services.local import local_cluster, make_survey

    cl, node = local_cluster(3, 40, 1, device=gpu_device, workdir=str(tmp_path))
    client = DrynxClient(node, device=gpu_device)
    secret = sum(cn.keypair.secret for cn in cl.cns) % O.R
    try:
        for op in ("variance", "lin_reg", "frequencyCount", "min"):
            sq = make_survey(client, cl, op, query_min=0, query_max=5, rows=50, d=3, proofs=1, ranges=[16, 16],
                             sig_device=gpu_device, deterministic_sigs=True)
            batch = dcp.dp_encode_batch(node, sq, list(cl.dps))
            for dp in list(cl.dps)[:5]:
                single = dcp.dp_encode(node, sq, dp)
                assert batch[dp.id]["clear"] == single["clear"], op
                assert eg.decrypt_ints(secret, batch[dp.id]["cv"]) == batch[dp.id]["clear"][0], op
    finally:
        node.close(remove=True)


@pytest.mark.parametrize("K", [1, 8])
def test_shared_v_fold_infinities(gpu_device, K):
    """Shared-V coefficients + per-verifier evaluation: items whose P or V is
    the point at infinity contribute 1, as in the per-item line image."""
    m, G = 700, 2
    period = -(-m // (64 * K * nt.FOLD_P_ALIGN)) * 64 * K * nt.FOLD_P_ALIGN
    V = nt.g2_fb_mul(bn.base2_table(gpu_device), bn.random_scalars(m, gpu_device))
    V[5] = 0
    V[640] = 0
    P = torch.zeros((G * period, 16), dtype=torch.int32, device=gpu_device)
    for v in range(G):
        Pv = nt.g1_to_affine(nt.g1_fb_mul(bn.base_table(gpu_device), bn.random_scalars(m, gpu_device)))
        Pv[3 + v] = 0
        P[v * period: v * period + m] = Pv
    fb = nt.rp_fold_accum_p(nt.rp_fold_coeffs(V), P, V, period, G, K)
    blk = period // (64 * K)
    for v in range(G):
        Pv = P[v * period: v * period + m].contiguous()
        alone = nt.rp_fold_accum(nt.rp_fold_lines(Pv, V), m, 1)
        a = nt.final_exp(nt._finish_prod_on_host(fb[v * blk:(v + 1) * blk]))
        b = nt.final_exp(nt._finish_prod_on_host(alone))
        assert bool(nt.gt_eq(a, b).all()), v


def test_gpu_ops_match_oracle(gpu_device):
    """GT exponentiation, G2 scalar multiplication and the G1 MSM on gfx950
    against the pure-Python oracle (not the native host path)."""
    ks = [RNG.randrange(O.R) for _ in range(6)] + [0, 1, O.R - 1]
    kt = bn.scalars_tensor(ks, gpu_device)
    e = O.pairing(O.G1_GEN, O.G2_GEN)
    g = nt.gt_pow(bn.gt_tensor([e], gpu_device), kt).cpu()
    assert bn.gt_from_tensor(g) == [e ** k for k in ks]
    q = O.g2_mul(7, O.G2_GEN)
    g2 = nt.g2_mul(bn.g2_aff_tensor([q], gpu_device), kt).cpu()
    assert bn.g2_points_from_aff(g2) == [None if k % O.R == 0 else O.g2_mul(k, q) for k in ks]
    g2 = nt.g2_fb_mul(bn.base2_table(gpu_device), kt).cpu()
    assert bn.g2_points_from_aff(g2) == [None if k % O.R == 0 else O.g2_mul(k, O.G2_GEN) for k in ks]
    pts = [O.g1_mul(RNG.randrange(1, O.R), O.G1_GEN) for _ in range(300)]
    sc = [RNG.randrange(O.R) for _ in range(300)]
    got = nt.g1_msm(bn.g1_jac_tensor(pts, gpu_device), bn.scalars_tensor(sc, gpu_device))
    exp = None
    for p, k in zip(pts, sc):
        exp = O.g1_add(exp, O.g1_mul(k, p))
    assert bn.g1_points_from_jac(got)[0] == exp


def test_glv_points_match_host(gpu_device):
    """GLV point kernel == affine((a + b lambda)(ZB - Y)) computed with the
    host path's full-scalar multiplication, incl. T at infinity."""
    S, L, npj = 2, 3, 9
    ZB = nt.g1_fb_mul(bn.base_table(gpu_device), bn.random_scalars(npj * L, gpu_device))
    Y = nt.g1_fb_mul(bn.base_table(gpu_device), bn.random_scalars(npj * S, gpu_device))
    Y[1] = ZB[0]  # T = ZB - Y = infinity for every item of (p=0, i=1, j=0)
    m = npj * S * L
    ab, rho = nt.glv_weights(m, gpu_device)
    got = nt.rp_fold_points_glv(ZB, Y, ab, S, L).cpu()
    zb = ZB.cpu().view(npj, 1, L, 24).expand(npj, S, L, 24).reshape(-1, 24).contiguous()
    yy = Y.cpu().view(npj, S, 1, 24).expand(npj, S, L, 24).reshape(-1, 24).contiguous()
    T = nt.g1_add(zb, yy, subtract=True)
    exp = nt.g1_to_affine(nt.g1_mul(T, rho.cpu()))
    assert torch.equal(got, exp)


@pytest.mark.parametrize("K", [1, 8])
def test_normalised_fold_matches_shared_v(gpu_device, K):
    """Fold mode 4 (lines normalised to 1 + (a u) w + (b v) w^3) == mode 3
    after the final exponentiation, with points / V at infinity."""
    m, G = 700, 2
    period = -(-m // (64 * K * nt.FOLD_P_ALIGN)) * 64 * K * nt.FOLD_P_ALIGN
    V = nt.g2_fb_mul(bn.base2_table(gpu_device), bn.random_scalars(m, gpu_device))
    V[7] = 0
    P = torch.zeros((G * period, 16), dtype=torch.int32, device=gpu_device)
    for v in range(G):
        Pv = nt.g1_to_affine(nt.g1_fb_mul(bn.base_table(gpu_device), bn.random_scalars(m, gpu_device)))
        Pv[11 + v] = 0
        P[v * period: v * period + m] = Pv
    ref = nt.rp_fold_accum_p(nt.rp_fold_coeffs(V), P, V, period, G, K)
    UV = nt.g1_aff_to_uv_(P.clone())
    got = nt.rp_fold_accum_n(nt.rp_fold_ncoeffs(V), UV, V, period, G, K)
    blk = period // (64 * K)
    for v in range(G):
        a = nt.final_exp(nt._finish_prod_on_host(got[v * blk:(v + 1) * blk]))
        b = nt.final_exp(nt._finish_prod_on_host(ref[v * blk:(v + 1) * blk]))
        assert bool(nt.gt_eq(a, b).all()), v


def test_ufold_coop_matches_one_lane(gpu_device):
    """The three-lanes-per-item U-side accumulation over raw line
    coefficients (dx_ufold_coop.hip) == the one-lane normalised rp_accum_n
    kernel block by block after the final exponentiation (normalising the
    lines changes the Miller value by a factor the final exponentiation
    kills), with points / V at infinity and padding."""
    m, G = 700, 2
    period = -(-m // (64 * nt.FOLD_P_ALIGN)) * 64 * nt.FOLD_P_ALIGN
    V = nt.g2_fb_mul(bn.base2_table(gpu_device), bn.random_scalars(m, gpu_device))
    V[7] = 0
    P = torch.zeros((G * period, 16), dtype=torch.int32, device=gpu_device)
    for v in range(G):
        Pv = nt.g1_to_affine(nt.g1_fb_mul(bn.base_table(gpu_device), bn.random_scalars(m, gpu_device)))
        Pv[11 + v] = 0
        P[v * period: v * period + m] = Pv
    got = nt.rp_fold_accum_coop_raw(nt.rp_fold_coeffs(V), P, V, period, G)
    ref = nt.rp_fold_accum_n(nt.rp_fold_ncoeffs(V), nt.g1_aff_to_uv_(P.clone()), V, period, G, 1)
    assert got.shape == ref.shape
    assert bool(nt.gt_eq(nt.final_exp(got.cpu()), nt.final_exp(ref.cpu())).all())


def test_copy_to_host_small_grid(gpu_device):
    """The ledger's device-to-host payload copy (nt.copy_to_host, a 32-block
    persistent grid writing pinned host memory) == the device bytes, for
    regions of odd word counts at 4-byte offsets (interior views included)."""
    g = torch.Generator(device=gpu_device).manual_seed(5)
    words = [1, 7, 4096, 4097, 70001, 1 << 20]
    src = [torch.randint(-2 ** 31, 2 ** 31 - 1, (w + 3,), generator=g, device=gpu_device, dtype=torch.int64)
           .to(torch.int32)[3:] for w in words]                                # 12-byte offset views
    total = sum(4 * w for w in words)
    host = torch.empty(total + 64, dtype=torch.uint8, pin_memory=True)
    pairs, o = [], 4
    for t in src:
        b = t.view(torch.uint8)
        pairs.append((b, host[o: o + b.numel()]))
        o += b.numel()
    nt.copy_to_host(pairs, host)
    torch.cuda.synchronize()
    for t, (_, h) in zip(src, pairs):
        assert torch.equal(h.view(torch.int32), t.cpu())
