"""Range-proof verification by bilinearity (verifier mode "msm",
csrc/kernels/dx_rpmsm.hip): the G2 joint table, the L-point combinations
U, the Pippenger G2 MSM and the regrouped pairing product, each against the
pure-Python oracle (host path here, the gfx950 kernels under -m gpu), the
device-resident bucket plans (no host sync) against the oracle, and the
regrouped pairing product against the per-item Miller product on the same
proofs."""
import random

import pytest
import torch

from drynx_amd import native as nt
from drynx_amd.crypto import bn254 as bn
from drynx_amd.crypto import elgamal as eg
from drynx_amd.crypto import oracle as O
from drynx_amd.ops.encoding import CreateProofBatch
from drynx_amd.proofs import range_proof as rp

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _dev(name):
    if name == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device(name)


def _g2_points(k, seed):
    rnd = random.Random(seed)
    return [O.g2_mul(rnd.randrange(1, O.R), O.G2_GEN) for _ in range(k)]


def _lam_mul(a: int, b: int, Q):
    return O.g2_mul((a + b * nt.GLV_LAMBDA) % O.R, Q)


@pytest.mark.parametrize("device", DEVICES)
def test_joint_table_entries(device):
    dev = _dev(device)
    pts = _g2_points(3, 1) + [None]                       # None = infinity row
    V = bn.g2_aff_tensor(pts, dev)
    T = bn.g2_points_from_aff(nt.g2_joint_table(V).cpu())
    for i, Q in enumerate(pts):
        for e in range(15):
            da, db = (e + 1) % 4, (e + 1) // 4
            want = None if Q is None else _lam_mul(da, db, Q)
            assert T[i * 15 + e] == want, (i, da, db)


@pytest.mark.parametrize("device", DEVICES)
def test_u_joint_combinations(device):
    dev = _dev(device)
    G, nq, L = 2, 3, 4
    pts = _g2_points(nq * L, 2)
    pts[5] = None                                         # an infinity V inside a group
    V = bn.g2_aff_tensor(pts, dev)
    rnd = random.Random(3)
    ab = [[rnd.getrandbits(32), rnd.getrandbits(32)] for _ in range(G * nq * L)]
    ab[0] = [0, 0]
    ab_t = torch.tensor(ab, dtype=torch.int64).to(torch.int32).to(dev)
    pad = nq + 2
    out = torch.zeros((G * pad, 32), dtype=torch.int32, device=dev)
    nt.rp_u_joint(nt.g2_joint_table(V), ab_t, nq, G, L, out, pad)
    got = bn.g2_points_from_aff(out.cpu())
    for v in range(G):
        for q in range(nq):
            acc = None
            for j in range(L):
                Q = pts[q * L + j]
                if Q is not None:
                    a, b = ab[(v * nq + q) * L + j]
                    acc = O.g2_add(acc, _lam_mul(a, b, Q))
            assert got[v * pad + q] == acc, (v, q)
        assert got[v * pad + nq] is None                  # untouched rows stay infinity
    # an explicit row per (v, q) (the segmented fold layout): the same points, permuted
    perm = list(range(G * pad))
    random.Random(9).shuffle(perm)
    pos = torch.tensor(perm[: G * nq], dtype=torch.int64, device=dev)
    out2 = torch.zeros((G * pad, 32), dtype=torch.int32, device=dev)
    nt.rp_u_joint(nt.g2_joint_table(V), ab_t, nq, G, L, out2, pad, pos)
    want = out.view(G, pad, 32)[:, :nq].reshape(-1, 32)
    assert torch.equal(out2.index_select(0, pos), want)


@pytest.mark.gpu
@pytest.mark.parametrize("L", [16, 5])
def test_u_joint_split_matches_host(L):
    """Pool-slice sizes split each (v, q) over 4 lanes reduced through LDS in
    the same workgroup (u_joint_fused_kernel): many workgroups, groups of
    lanes whose digit ranges are uneven or empty (L = 5), against the host
    path (separate partials + reduction)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    G, nq = 3, 50
    rnd = random.Random(11)
    base = _g2_points(7, 4)
    pts = [base[rnd.randrange(7)] for _ in range(nq * L)]  # repeated points: doubling cases in the sums
    V = bn.g2_aff_tensor(pts, "cpu")
    ab = torch.tensor([[rnd.getrandbits(32), rnd.getrandbits(32)] for _ in range(G * nq * L)],
                      dtype=torch.int64).to(torch.int32)
    pad = nq + 3
    outs = []
    for dev in ("cpu", "cuda"):
        out = torch.zeros((G * pad, 32), dtype=torch.int32, device=dev)
        nt.rp_u_joint(nt.g2_joint_table(V.to(dev)), ab.to(dev), nq, G, L, out, pad)
        outs.append(out.cpu())
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("c", [13, 4])
def test_g2_msm_grouped(device, c):
    dev = _dev(device)
    m, G = 11, 3
    pts = _g2_points(m, 4)
    V = bn.g2_aff_tensor(pts, dev)
    rnd = random.Random(5)
    ks = [rnd.randrange(O.R) for _ in range(G * m)]
    ks[2] = 0
    ks[7] = O.R - 1
    k = bn.scalars_tensor(ks, dev)
    grp = torch.arange(G, dtype=torch.int32, device=dev).repeat_interleave(m)
    h = nt.g2_msm_launch(V, k, grp, G, c=c)
    stride, off = 4, 1
    out = torch.zeros((G * stride, 32), dtype=torch.int32, device=dev)
    nt.g2_msm_finish(nt.g2_msm_run(V, h), h, out, stride, off)     # device Horner lanes
    assert bn.g2_points_from_aff(nt.g2_msm_finish(nt.g2_msm_run(V, h).cpu(), h).cpu()) == \
        [bn.g2_points_from_aff(out.cpu())[g * stride + off] for g in range(G)]   # host Horner
    got = bn.g2_points_from_aff(out.cpu())
    for g in range(G):
        want = None
        for t in range(m):
            want = O.g2_add(want, O.g2_mul(ks[g * m + t], pts[t]))
        assert got[g * stride + off] == want, g


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("skew", [False, True])
def test_g2_msm_device_plan(device, skew):
    """Device-resident plan (csrc/kernels/dx_plan.hip dx_lane_slices): lanes
    per bucket fixed by the shape; skewed scalars (every entry in one bucket
    per window) only lengthen the lanes' slices."""
    dev = _dev(device)
    m, G, c = 13, 2, 4
    pts = _g2_points(m, 6)
    pts[3] = None
    V = bn.g2_aff_tensor(pts, dev)
    rnd = random.Random(7)
    ks = [(0x123456789 if skew else rnd.randrange(O.R)) for _ in range(G * m)]
    ks[5] = 0
    S, h = nt.g2_msm_device(V, bn.scalars_tensor(ks, dev), m, ((m, 254),) * G, c=c)
    got = bn.g2_points_from_aff(nt.g2_msm_finish(S.cpu(), h).cpu())
    nt.check_overflow(h)
    for g in range(G):
        want = None
        for t in range(m):
            if pts[t] is not None:
                want = O.g2_add(want, O.g2_mul(ks[g * m + t], pts[t]))
        assert got[g] == want, g


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("wc", [(4, 11), (3, 16)])
def test_multi_exp_and_g1_msm_device_plans(device, wc):
    """GT multi-exponentiation (two groups of different exponent widths,
    two row periods) and the G1 MSM with device-resident plans against the
    oracle; an exponent wider than declared is reported, not dropped silently."""
    dev = _dev(device)
    rnd = random.Random(9)
    n = 5
    a_pts = [O.pairing(O.g1_mul(rnd.randrange(1, O.R), O.G1_GEN), O.G2_GEN) for _ in range(n)]
    a = bn.gt_tensor(a_pts, dev)
    e32 = [rnd.getrandbits(32) for _ in range(2 * n)]   # group 0: rows i < 2n over a[i % n]
    e40 = [rnd.getrandbits(40) for _ in range(n)]       # group 1: rows over a[(i - 2n) % n]
    k = torch.zeros((3 * n, 8), dtype=torch.int64)
    for i, e in enumerate(e32 + e40):
        k[i, 0], k[i, 1] = e & 0xffffffff, e >> 32
    k = k.to(torch.int32).to(dev)
    grp = torch.tensor([0] * (2 * n) + [1] * n, dtype=torch.int32, device=dev)
    h = nt.multi_exp_device(a, k, grp, ((2 * n, 32), (n, 40)), *wc, item_split=(2 * n, n))
    got = nt.multi_exp_grouped_finish(h)
    nt.check_overflow(h)
    def pw(x, e):
        r, b = O.Fp12.one(), x
        while e:
            if e & 1:
                r = r * b
            b, e = b * b, e >> 1
        return r

    want0, want1 = O.Fp12.one(), O.Fp12.one()
    for i in range(2 * n):
        want0 = want0 * pw(a_pts[i % n], e32[i])
    for i in range(n):
        want1 = want1 * pw(a_pts[i], e40[i])
    assert bn.gt_from_tensor(got.cpu()) == [want0, want1]
    # an exponent wider than group 0's declared 32 bits
    k2 = k.clone()
    k2[0, 1] = 1
    h2 = nt.multi_exp_device(a, k2, grp, ((2 * n, 32), (n, 40)), *wc, item_split=(2 * n, n))
    nt.multi_exp_grouped_finish(h2)
    with pytest.raises(RuntimeError, match="declared scalar widths"):
        nt.check_overflow(h2)
    # G1: two groups of 254-bit scalars
    pts = [O.g1_mul(rnd.randrange(1, O.R), O.G1_GEN) for _ in range(6)]
    ks = [rnd.randrange(O.R) for _ in range(12)]
    P = bn.g1_jac_tensor(pts + pts, dev)
    hd = nt.g1_msm_device(P, bn.scalars_tensor(ks, dev), 6, ((6, 254), (6, 254)))
    got = nt.g1_msm_finish(hd)
    nt.check_overflow(hd)
    for g in range(2):
        want = None
        for t in range(6):
            want = O.g1_add(want, O.g1_mul(ks[g * 6 + t], pts[t]))
        assert bn.g1_points_from_jac(got[g: g + 1])[0] == want, g


@pytest.fixture(scope="module")
def proofs():
    S, u, l = 2, 4, 3
    sigs = [[rp.init_range_proof_signature(u) for _ in range(3)] for _ in range(S)]
    kps = [eg.KeyPair.generate() for _ in range(S)]
    P = eg.aggregate_keys([k.public for k in kps])
    sm = rp.SigMaterial(sigs)
    vals = [0, 17, 63, 5]
    cv, r = eg.encrypt_ints(eg.pk_table(P), vals)
    n = len(vals)
    b = CreateProofBatch(vals, r, cv, [u] * n, [l] * n, [0, 1, 2, 0], [0] * n)
    return rp.create_range_proofs(b, sm, P)[0], sm, P


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("segs", [None, [1, 2, 1]])
def test_msm_pairing_product_matches_per_item_fold(device, proofs, segs):
    """FE(ML(B, R) prod ML(-Y_q, U_q)) == FE(prod_it ML(rho (Zphi B - Y), V_it))
    for the same weights: the regrouping is an identity, not a new check."""
    dev = _dev(device)
    rpl, sm, _ = proofs
    r = rpl.to(dev)
    n, l, S = len(r), r.l, r.S
    m, G = n * S * l, 2
    ZB = nt.g1_fb_mul(bn.base_table(dev), r.zphi)
    y_idx = (torch.arange(S, device=dev).view(1, S) * sm.n_cols
             + torch.tensor(r.cols, device=dev).view(n, 1)).reshape(-1)
    Y = nt.g1_mul(sm.y_jac.to(dev).index_select(0, y_idx).contiguous(), rp._rep(r.challenge, S))
    ab, rho = nt.glv_weights(G * m, dev)
    it = torch.arange(m, device=dev)
    s_r = nt.fr_arith(nt.FR_MUL, rho, r.zphi.index_select(0, (it // (S * l)) * l + it % l).contiguous())
    S_R, hR = nt.g2_msm_device(r.V, s_r, m, ((m, 254),) * G, c=rp._r_window(m, G))
    q = rp._msm_queue(Y, r.V, ab, G, n, S, l, None, segs)
    fR, _ = rp._msm_r_miller(hR, S_R)
    useg = rp._seg_products(q)                            # per (VN, segment) U-side products
    k = len(segs) if segs else 1
    assert tuple(useg.shape) == (G, k, 96)
    # T_it = Zphi_(p,j) B - Y_(p,i) for item it = (p S + i) L + j
    zb = ZB.cpu().view(n, 1, l, 24).expand(n, S, l, 24).reshape(-1, 24)
    yy = Y.cpu().view(n, S, 1, 24).expand(n, S, l, 24).reshape(-1, 24)
    T = nt.g1_add(zb.contiguous(), yy.contiguous(), subtract=True)
    for v in range(G):
        F_msm = nt.gt_mul(nt.gt_prod(useg[v].view(k, 1, 96), chunk=4).view(1, 96), fR[v:v + 1])
        f = nt.miller_loop(nt.g1_to_affine(nt.g1_mul(T, rho[v * m:(v + 1) * m].cpu().contiguous())), r.V.cpu())
        F_fold = nt.gt_prod(f.view(-1, 1, 96), chunk=4).view(1, 96)
        assert bool(nt.gt_eq(nt.final_exp(F_msm.cpu()), nt.final_exp(F_fold)).all()), v


@pytest.mark.parametrize("device", DEVICES)
def test_verifier_accepts_and_rejects(device, proofs):
    dev = _dev(device)
    rpl, sm, P = proofs
    assert rp.verify_range_proof_list_multi(rpl.to(dev), sm, P, 3, dev) == [True] * 3
    bad = rpl.to(dev)
    V = bad.V.clone()
    V[4] = V[5]                                           # a valid G2 point, wrong item
    bad.V = V
    assert rp.verify_range_proof_list_multi(bad, sm, P, 2, dev) == [False] * 2


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("field", ["V", "zr", "A", "A_off_gt"])
def test_segment_attribution(device, field, proofs, monkeypatch):
    """segs = per-request slices: a clean batch clears every segment; a
    tampered proof is named by the failing VN's segment-grouped second pass
    (pairing side: V; D-equation: Zr; GT side: A), the other segments pass."""
    dev = _dev(device)
    rpl, sm, P = proofs
    r = rpl.to(dev)
    assert rp.verify_range_proof_list_multi(r, sm, P, 2, dev, segs=[1, 2, 1]) == [[True] * 3] * 2
    bad = rpl.to(dev)
    n, l, S = len(bad), bad.l, bad.S
    if field == "V":                                      # proof 2 (segment 1): a valid G2 point, wrong item
        V = bad.V.clone()
        V[2 * S * l] = V[2 * S * l + 1]
        bad.V = V
        want = [True, False, True]
    elif field == "zr":                                   # proof 3 (segment 2)
        zr = bad.zr.clone()
        zr[3, 0] ^= 1
        bad.zr = zr
        want = [True, True, False]
    elif field == "A":                                    # proof 0 (segment 0): a_it^2 is still in GT
        A = bad.A.clone()
        A[1] = nt.gt_mul(A[1:2].contiguous(), A[1:2].contiguous())[0]
        bad.A = A
        want = [False, True, True]
    else:                                                 # the last word flipped (FaultPlan corrupt_proof): off GT
        A = bad.A.clone()
        A[-1, -1] ^= 1
        bad.A = A
        want = [True, True, False]
    decodes = field != "A_off_gt"
    calls, hinted = [], []
    orig, orig_h = rp._segment_pass, rp._segment_hinted
    monkeypatch.setattr(rp, "_segment_pass", lambda *a: calls.append(1) or orig(*a))
    monkeypatch.setattr(rp, "_segment_hinted", lambda *a: hinted.append(orig_h(*a)) or hinted[-1])
    # the first failing VN's full segment pass, the others' verdicts from its
    # hint; a proof that does not decode gets zero weights: the batch of the
    # others passes, no second pass at all
    assert rp.verify_range_proof_list_multi(bad, sm, P, 3, dev, segs=[1, 2, 1]) == [want] * 3
    assert len(calls) == (3 if decodes else 0)       # one full pass + each hinted VN's pass over T
    assert len(hinted) == (2 if decodes else 0) and all(h == want for h in hinted)
    assert rp.verify_range_proof_list_multi(bad, sm, P, 2, dev) == [False] * 2


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("dmode", ["direct", "msm"])
def test_dcheck_direct_and_bucket_agree(device, dmode, proofs, monkeypatch):
    """The D-check as GLV ladders + tree sums (no bucket plan) and as the
    bucket MSM accept the same batch and reject a tampered Zr, with per-VN
    attribution."""
    dev = _dev(device)
    monkeypatch.setenv("DRYNX_DCHECK", dmode)
    rpl, sm, P = proofs
    assert rp.verify_range_proof_list_multi(rpl.to(dev), sm, P, 3, dev, segs=[1, 2, 1]) == [[True] * 3] * 3
    bad = rpl.to(dev)
    zr = bad.zr.clone()
    zr[1, 0] ^= 1
    bad.zr = zr
    assert rp.verify_range_proof_list_multi(bad, sm, P, 3, dev, segs=[1, 2, 1]) == [[True, False, True]] * 3
    assert rp.verify_range_proof_list_multi(bad, sm, P, 2, dev) == [False] * 2
