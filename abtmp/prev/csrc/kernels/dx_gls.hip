// GLS-2 fixed-base tables for the range-proof prover (K6/K7, table mode 6).
//
// The prover's per-item work is V = v A_phi (G2) and e(B, A_phi)^(-s v) (GT)
// with per-signature bases (lib/range/range_proof.go:452-469; here from comb
// tables instead of a pairing per item).  Both groups carry an endomorphism
// with eigenvalue lambda2 = 6u^2 = p (mod r), a ~127-bit number:
//   G2: psi(x, y) = (conj(x) w1, conj(y) w2)  (untwist-Frobenius-twist),
//   GT: x -> x^p (Frobenius).
// Any scalar k < r splits as k = k0 + k1 lambda2 with k0 < lambda2 and
// k1 < r / lambda2 < 2^128 by one long division (no lattice: lambda2 ~ sqrt r),
// so  k Q = k0 Q + psi(k1 Q)  and  x^k = x^k0 * frob(x^k1): two fixed-base
// evaluations over 132-bit exponents from ONE table per base.  With 6-bit
// windows a table holds 22 x 63 entries (1386: 177 KiB per G2 base, 532 KiB
// per GT base) and an evaluation costs 44 mixed additions / Fp12 products
// instead of the 64 of the 4-bit 256-bit comb (960 entries).
#include "common.h"

using namespace dxk;

namespace {
constexpr int kBits = 6;
constexpr int kDig = (1 << kBits) - 1;   // 63 non-zero digits
constexpr int kWin = 22;                 // 132 bits >= any half
constexpr int kEnt = kWin * kDig;        // 1386

// k (8 limbs) = k0 + k1 * lambda2, k0 < lambda2 (4 limbs), k1 < 2^130 (5 limbs):
// restoring binary long division by the 127-bit constant.
DX_HD void split_l2(const uint32_t *k, uint32_t *k0, uint32_t *k1) {
  uint32_t rem[5] = {0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int bit = 255; bit >= 0; bit--) {
#pragma unroll
    for (int i = 4; i > 0; i--) rem[i] = (rem[i] << 1) | (rem[i - 1] >> 31);
    rem[0] = (rem[0] << 1) | ((k[bit >> 5] >> (bit & 31)) & 1u);
    uint32_t d[5], br = 0;
#pragma unroll
    for (int i = 0; i < 5; i++) d[i] = subb32(rem[i], i < 4 ? SIX_U2[i] : 0u, br);
    if (!br) {  // rem >= lambda2
#pragma unroll
      for (int i = 0; i < 5; i++) rem[i] = d[i];
      q[bit >> 5] |= 1u << (bit & 31);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; i++) k0[i] = rem[i];
  k0[4] = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) k1[i] = q[i];
}

DX_HD uint32_t digit6(const uint32_t *k, int w) {
  const int bit = w * kBits;
  uint32_t v = k[bit >> 5] >> (bit & 31);
  if ((bit & 31) + kBits > 32 && (bit >> 5) + 1 < 5) v |= k[(bit >> 5) + 1] << (32 - (bit & 31));
  return v & (uint32_t)kDig;
}

DX_HD G2J psi_jac(const G2J &q) {
  return {mul(conj(q.x), Fp2::from_limbs(Frob::TWX1)), mul(conj(q.y), Fp2::from_limbs(Frob::TWY1)), conj(q.z)};
}

DX_NI G2J g2_gls6_eval(const G2A *T, const uint32_t *k) {
  uint32_t k0[5], k1[5];
  split_l2(k, k0, k1);
  // one accumulator: psi(sum T[d1]) first, then the k0 digits on top
  G2J a = G2J::inf();
  for (int w = 0; w < kWin; w++) {
    const uint32_t d1 = digit6(k1, w);
    if (d1) a = jadd_mixed(a, T[w * kDig + d1 - 1]);
  }
  a = psi_jac(a);
  for (int w = 0; w < kWin; w++) {
    const uint32_t d0 = digit6(k0, w);
    if (d0) a = jadd_mixed(a, T[w * kDig + d0 - 1]);
  }
  return a;
}

DX_NI Fp12 gt_gls6_eval(const Fp12 *T, const uint32_t *k) {
  uint32_t k0[5], k1[5];
  split_l2(k, k0, k1);
  // one accumulator: frob(prod T[d1]) first, then the k0 digits on top
  Fp12 f = Fp12::one();
  for (int w = 0; w < kWin; w++) {
    const uint32_t d1 = digit6(k1, w);
    if (d1) f = mul(f, T[w * kDig + d1 - 1]);
  }
  f = frob<1>(f);
  for (int w = 0; w < kWin; w++) {
    const uint32_t d0 = digit6(k0, w);
    if (d0) f = mul(f, T[w * kDig + d0 - 1]);
  }
  return f;
}
}  // namespace

extern "C" {
int dx_gls6_entries() { return kEnt; }

// table[b*1386 + w*63 + d-1] = d 2^(6w) A_b (affine); work [nb*22] Jacobian
int dx_g2_gls6_table(int on_gpu, void *stream, const uint32_t *bases_aff, uint32_t *work, uint32_t *table,
                     int64_t n_bases) {
  auto p1 = [=] __host__ __device__(int64_t b) {
    G2J acc = G2J::from_aff(at<G2A>(bases_aff, b));
    for (int w = 0; w < kWin; w++) {
      at<G2J>(work, b * kWin + w) = acc;
      for (int i = 0; i < kBits; i++) acc = jdbl(acc);
    }
  };
  int rc = run(on_gpu, stream, n_bases, p1, true, "g2_gls6_pow64");
  if (rc) return rc;
  auto p2 = [=] __host__ __device__(int64_t t) {
    const int64_t b = t / kEnt, i = t % kEnt;
    const int w = (int)(i / kDig), d = (int)(i % kDig) + 1;
    const G2J q = at<G2J>(work, b * kWin + w);
    G2J acc = G2J::inf();
    for (int bit = kBits - 1; bit >= 0; bit--) {
      acc = jdbl(acc);
      if ((d >> bit) & 1) acc = jadd(acc, q);
    }
    at<G2A>(table, t) = to_affine(acc);
  };
  return run(on_gpu, stream, n_bases * kEnt, p2, true, "g2_gls6_table");
}

int dx_g2_gls6_mul(int on_gpu, void *stream, const uint32_t *tables, const int32_t *tab_idx, const uint32_t *scalars,
                   uint32_t *out_aff, int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) {
    const G2A *T = reinterpret_cast<const G2A *>(tables) + (int64_t)(tab_idx ? tab_idx[i] : 0) * kEnt;
    at<G2A>(out_aff, i) = to_affine(g2_gls6_eval(T, scalars + 8 * i));
  };
  return run(on_gpu, stream, n, op, true, "g2_gls6_mul");
}

// table[b*1386 + w*63 + d-1] = E_b^(d 2^(6w)); work [nb*22]
int dx_gt_gls6_table(int on_gpu, void *stream, const uint32_t *bases, uint32_t *work, uint32_t *table,
                     int64_t n_bases) {
  auto p1 = [=] __host__ __device__(int64_t b) {
    Fp12 acc = at<Fp12>(bases, b);
    for (int w = 0; w < kWin; w++) {
      at<Fp12>(work, b * kWin + w) = acc;
      for (int i = 0; i < kBits; i++) acc = cyclotomic_sqr(acc);
    }
  };
  int rc = run(on_gpu, stream, n_bases, p1, true, "gt_gls6_pow64");
  if (rc) return rc;
  auto p2 = [=] __host__ __device__(int64_t t) {
    const int64_t b = t / kEnt, i = t % kEnt;
    const int w = (int)(i / kDig), d = (int)(i % kDig) + 1;
    const Fp12 q = at<Fp12>(work, b * kWin + w);
    Fp12 acc = Fp12::one();
    for (int bit = kBits - 1; bit >= 0; bit--) {
      acc = cyclotomic_sqr(acc);
      if ((d >> bit) & 1) acc = mul(acc, q);
    }
    at<Fp12>(table, t) = acc;
  };
  return run(on_gpu, stream, n_bases * kEnt, p2, true, "gt_gls6_table");
}

int dx_gt_gls6_pow(int on_gpu, void *stream, const uint32_t *tables, const int32_t *tab_idx, const uint32_t *scalars,
                   uint32_t *out, int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) {
    const Fp12 *T = reinterpret_cast<const Fp12 *>(tables) + (int64_t)(tab_idx ? tab_idx[i] : 0) * kEnt;
    at<Fp12>(out, i) = gt_gls6_eval(T, scalars + 8 * i);
  };
  return run(on_gpu, stream, n, op, true, "gt_gls6_pow");
}

// a[it] = E_phi(it)^(e[it]) * gT^(t[p, j]) with the GLS-6 tables (the shared
// gT^t part as dx_rp_prove_a_tab: computed once per (p, j) in a first pass).
int dx_rp_prove_a_gls6(int on_gpu, void *stream, const uint32_t *gphi_tables, const int32_t *tab_idx,
                       const uint32_t *e_sc, const uint32_t *t_sc, const uint32_t *gt_table, uint32_t *a_out,
                       int64_t n_items, int S, int L) {
  const int64_t n_pj = n_items / S;
  auto p1 = [=] __host__ __device__(int64_t pj) {
    const int64_t p = pj / L, j = pj % L;
    at<Fp12>(a_out, p * S * L + j) = gt_fixed_pow(reinterpret_cast<const Fp12 *>(gt_table), t_sc + 8 * pj);
  };
  int rc = run(on_gpu, stream, n_pj, p1, true, "rp_prove_gt_t");
  if (rc) return rc;
  for (int pass = 0; pass < 2; pass++) {
    const int64_t per = pass == 0 ? (int64_t)(S - 1) * L : (int64_t)L;
    if (per == 0) continue;
    const int64_t n = n_pj / L * per;
    auto p2 = [=] __host__ __device__(int64_t k) {
      const int64_t p = k / per, r = k % per;
      const int64_t i = pass == 0 ? 1 + r / L : 0, j = r % L;
      const int64_t it = (p * S + i) * L + j;
      const Fp12 *T = reinterpret_cast<const Fp12 *>(gphi_tables) + (int64_t)tab_idx[it] * kEnt;
      at<Fp12>(a_out, it) = mul(gt_gls6_eval(T, e_sc + 8 * it), at<Fp12>(a_out, p * S * L + j));
    };
    rc = run(on_gpu, stream, n, p2, true, "rp_prove_a_gls6");
    if (rc) return rc;
  }
  return 0;
}
}  // extern "C"
