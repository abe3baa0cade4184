// BN254 G1 (over Fp) and G2 (D-type twist over Fp2) in Jacobian coordinates,
// a = 0.  One template serves both groups (field ops are overloaded).
// Replaces kyber bn256 curvePoint/twistPoint (external; used across the
// reference via libunlynx.SuiTe.Point(), e.g. lib/range/range_proof.go:383-398).
//
// Storage conventions shared with the Python side (drynx_amd/native):
//   Affine   G1 = 16 u32 (x, y) Montgomery, infinity = all zero.
//   Jacobian G1 = 24 u32 (X, Y, Z) Montgomery, infinity <=> Z == 0.
//   G2 doubles every coordinate (Fp2 = 16 u32).
//   Scalars are 8 u32 little-endian canonical integers (< r).
#pragma once
#include "tower.h"

namespace dx {

// Uniform field-op names for the curve template.
template <class PR> DX_HD FieldT<PR> add(const FieldT<PR> &a, const FieldT<PR> &b) { return fadd(a, b); }
template <class PR> DX_HD FieldT<PR> sub(const FieldT<PR> &a, const FieldT<PR> &b) { return fsub(a, b); }
template <class PR> DX_HD FieldT<PR> mul(const FieldT<PR> &a, const FieldT<PR> &b) { return fmul(a, b); }
template <class PR> DX_HD FieldT<PR> sqr(const FieldT<PR> &a) { return fsqr(a); }
template <class PR> DX_HD FieldT<PR> dbl(const FieldT<PR> &a) { return fdbl(a); }
template <class PR> DX_HD FieldT<PR> neg(const FieldT<PR> &a) { return fneg(a); }
template <class PR> DX_HD FieldT<PR> inv(const FieldT<PR> &a) { return finv(a); }
DX_HD bool fis_zero(const Fp &a) { return a.is_zero(); }
DX_HD bool fis_zero(const Fp2 &a) { return a.is_zero(); }
template <class F> DX_HD F fzero();
template <> DX_HD Fp fzero<Fp>() { return Fp::zero(); }
template <> DX_HD Fp2 fzero<Fp2>() { return Fp2::zero(); }
template <class F> DX_HD F fone();
template <> DX_HD Fp fone<Fp>() { return Fp::one(); }
template <> DX_HD Fp2 fone<Fp2>() { return Fp2::one(); }

template <class F>
struct Aff {
  F x, y;
  DX_HD bool is_inf() const { return fis_zero(x) && fis_zero(y); }
  static DX_HD Aff inf() { return {fzero<F>(), fzero<F>()}; }
};

template <class F>
struct Jac {
  F x, y, z;
  DX_HD bool is_inf() const { return fis_zero(z); }
  static DX_HD Jac inf() { return {fone<F>(), fone<F>(), fzero<F>()}; }
  static DX_HD Jac from_aff(const Aff<F> &a) {
    if (a.is_inf()) return inf();
    return {a.x, a.y, fone<F>()};
  }
};

using G1A = Aff<Fp>;
using G1J = Jac<Fp>;
using G2A = Aff<Fp2>;
using G2J = Jac<Fp2>;

// dbl-2009-l
template <class F>
DX_NI Jac<F> jdbl(const Jac<F> &p) {
  if (p.is_inf()) return p;
  F A = sqr(p.x), B = sqr(p.y), C = sqr(B);
  F D = dbl(sub(sub(sqr(add(p.x, B)), A), C));
  F E = add(dbl(A), A);
  F Fv = sqr(E);
  Jac<F> r;
  r.x = sub(Fv, dbl(D));
  F C8 = dbl(dbl(dbl(C)));
  r.y = sub(mul(E, sub(D, r.x)), C8);
  r.z = dbl(mul(p.y, p.z));
  return r;
}

// add-2007-bl with the exceptional cases handled.
template <class F>
DX_NI Jac<F> jadd(const Jac<F> &p, const Jac<F> &q) {
  if (p.is_inf()) return q;
  if (q.is_inf()) return p;
  F Z1Z1 = sqr(p.z), Z2Z2 = sqr(q.z);
  F U1 = mul(p.x, Z2Z2), U2 = mul(q.x, Z1Z1);
  F S1 = mul(mul(p.y, q.z), Z2Z2), S2 = mul(mul(q.y, p.z), Z1Z1);
  F H = sub(U2, U1);
  F rr = dbl(sub(S2, S1));
  if (fis_zero(H)) {
    if (fis_zero(rr)) return jdbl(p);
    return Jac<F>::inf();
  }
  F I = sqr(dbl(H));
  F J = mul(H, I);
  F V = mul(U1, I);
  Jac<F> r;
  r.x = sub(sub(sqr(rr), J), dbl(V));
  r.y = sub(mul(rr, sub(V, r.x)), dbl(mul(S1, J)));
  r.z = mul(sub(sub(sqr(add(p.z, q.z)), Z1Z1), Z2Z2), H);
  return r;
}

// madd-2007-bl: Jacobian + affine.
template <class F>
DX_NI Jac<F> jadd_mixed(const Jac<F> &p, const Aff<F> &q) {
  if (q.is_inf()) return p;
  if (p.is_inf()) return Jac<F>::from_aff(q);
  F Z1Z1 = sqr(p.z);
  F U2 = mul(q.x, Z1Z1);
  F S2 = mul(mul(q.y, p.z), Z1Z1);
  F H = sub(U2, p.x);
  F rr = dbl(sub(S2, p.y));
  if (fis_zero(H)) {
    if (fis_zero(rr)) return jdbl(p);
    return Jac<F>::inf();
  }
  F HH = sqr(H);
  F I = dbl(dbl(HH));
  F J = mul(H, I);
  F V = mul(p.x, I);
  Jac<F> r;
  r.x = sub(sub(sqr(rr), J), dbl(V));
  r.y = sub(mul(rr, sub(V, r.x)), dbl(mul(p.y, J)));
  r.z = sub(sub(sqr(add(p.z, H)), Z1Z1), HH);
  return r;
}

template <class F>
DX_HD Jac<F> jneg(const Jac<F> &p) {
  return {p.x, neg(p.y), p.z};
}
template <class F>
DX_HD Aff<F> aneg(const Aff<F> &p) {
  if (p.is_inf()) return p;
  return {p.x, neg(p.y)};
}

template <class F>
DX_NI Aff<F> to_affine(const Jac<F> &p) {
  if (p.is_inf()) return Aff<F>::inf();
  F zi = inv(p.z);
  F zi2 = sqr(zi);
  return {mul(p.x, zi2), mul(mul(p.y, zi2), zi)};
}

template <class F>
DX_HD bool jeq(const Jac<F> &p, const Jac<F> &q) {
  if (p.is_inf() || q.is_inf()) return p.is_inf() && q.is_inf();
  F Z1Z1 = sqr(p.z), Z2Z2 = sqr(q.z);
  if (!(mul(p.x, Z2Z2) == mul(q.x, Z1Z1))) return false;
  return mul(mul(p.y, q.z), Z2Z2) == mul(mul(q.y, p.z), Z1Z1);
}

DX_HD bool on_curve(const G1A &a) {
  if (a.is_inf()) return true;
  return fsqr(a.y) == fadd(fmul(fsqr(a.x), a.x), Fp::from_limbs(Curve::B1));
}
DX_HD bool on_curve(const G2A &a) {
  if (a.is_inf()) return true;
  return sqr(a.y) == add(mul(sqr(a.x), a.x), Fp2::from_limbs(Curve::B2));
}

DX_HD G1A g1_generator() { return {Fp::from_limbs(Curve::G1X), Fp::from_limbs(Curve::G1Y)}; }
DX_HD G2A g2_generator() { return {Fp2::from_limbs(Curve::G2X), Fp2::from_limbs(Curve::G2Y)}; }

DX_HD bool scalar_is_zero(const uint32_t *k) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) acc |= k[i];
  return acc == 0;
}

// Variable-base scalar multiplication: 4-bit fixed window, MSB first.
// The 16-entry window table lives in registers/scratch of the thread.
template <class F>
DX_NI Jac<F> scalar_mul(const Jac<F> &p, const uint32_t *k) {
  Jac<F> tab[16];
  tab[0] = Jac<F>::inf();
  tab[1] = p;
  for (int i = 2; i < 16; i++) tab[i] = (i & 1) ? jadd(tab[i - 1], p) : jdbl(tab[i >> 1]);
  Jac<F> r = Jac<F>::inf();
  int top = 63;  // skip leading zero windows (short scalars: 64-bit batch-verification weights)
  while (top > 0 && ((k[top >> 3] >> ((top & 7) * 4)) & 15u) == 0) top--;
  for (int w = top; w >= 0; w--) {
    r = jdbl(jdbl(jdbl(jdbl(r))));
    uint32_t d = (k[w >> 3] >> ((w & 7) * 4)) & 15u;
    if (d) r = jadd(r, tab[d]);
  }
  return r;
}

// Fixed-base comb: table[w*256 + d] = d * 2^(8w) * base (affine), w < 32.
// k*base = sum_w table[w][byte_w(k)]: 32 mixed additions, no doublings.
template <class F>
DX_NI Jac<F> fixed_base_mul(const Aff<F> *table, const uint32_t *k) {
  Jac<F> r = Jac<F>::inf();
#pragma unroll 4
  for (int w = 0; w < 32; w++) {
    uint32_t d = (k[w >> 2] >> ((w & 3) * 8)) & 255u;
    if (d) r = jadd_mixed(r, table[w * 256 + d]);
  }
  return r;
}

// Fixed-base comb with 4-bit windows: table[w*15 + d - 1] = d * 16^w * base
// (affine, d = 1..15, w < 64): 64 mixed additions, 120 KiB per G2 base.  The
// HBM-sized variant for large sets of distinct bases (one table per distinct
// Boneh-Boyen signature point of a query: 3 CNs x 2070 columns x u=16).
template <class F>
DX_NI Jac<F> fixed_base_mul4(const Aff<F> *table, const uint32_t *k) {
  Jac<F> r = Jac<F>::inf();
#pragma unroll 2
  for (int w = 0; w < 64; w++) {
    uint32_t d = (k[w >> 3] >> ((w & 7) * 4)) & 15u;
    if (d) r = jadd_mixed(r, table[w * 15 + d - 1]);
  }
  return r;
}

}  // namespace dx
