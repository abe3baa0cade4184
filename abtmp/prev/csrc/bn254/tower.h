// BN254 extension tower: Fp2 = Fp[i]/(i^2+1), Fp6 = Fp2[v]/(v^3-xi), xi = 9+i,
// Fp12 = Fp6[w]/(w^2-v).  Identical to drynx_amd/crypto/oracle.py so values
// compare coefficient for coefficient.  GT of the reference (kyber bn256
// gfP12, used by lib/range/range_proof.go:396-397,540-546) lives here.
#pragma once
#include "field.h"

namespace dx {

struct Fp2 {
  Fp c0, c1;
  static DX_HD Fp2 zero() { return {Fp::zero(), Fp::zero()}; }
  static DX_HD Fp2 one() { return {Fp::one(), Fp::zero()}; }
  static DX_HD Fp2 from_limbs(const uint32_t (*p)[8]) { return {Fp::from_limbs(p[0]), Fp::from_limbs(p[1])}; }
  DX_HD bool is_zero() const { return c0.is_zero() && c1.is_zero(); }
  DX_HD bool operator==(const Fp2 &o) const { return c0 == o.c0 && c1 == o.c1; }
};

DX_HD Fp2 add(const Fp2 &a, const Fp2 &b) { return {fadd(a.c0, b.c0), fadd(a.c1, b.c1)}; }
DX_HD Fp2 sub(const Fp2 &a, const Fp2 &b) { return {fsub(a.c0, b.c0), fsub(a.c1, b.c1)}; }
DX_HD Fp2 neg(const Fp2 &a) { return {fneg(a.c0), fneg(a.c1)}; }
DX_HD Fp2 dbl(const Fp2 &a) { return {fdbl(a.c0), fdbl(a.c1)}; }
DX_HD Fp2 conj(const Fp2 &a) { return {a.c0, fneg(a.c1)}; }
DX_HD Fp2 mul(const Fp2 &a, const Fp2 &b) {
#ifdef __HIP_DEVICE_COMPILE__
  // Karatsuba with lazy reduction: three 512-bit products, two reductions.
  //   c1 = (a0+a1)(b0+b1) - a0 b0 - a1 b1 = a0 b1 + a1 b0 < 2p^2
  //   c0 = a0 b0 - a1 b1 (+ p 2^256 if negative: the reduction maps it to +p)
  // Every reduction input is < p 2^256 (p < 2^254), as fred_wide requires.
  uint32_t sa[8], sb[8], T0[16], T1[16], T2[16];
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) sa[i] = addc32(a.c0.v[i], a.c1.v[i], c);
  c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) sb[i] = addc32(b.c0.v[i], b.c1.v[i], c);
  fmul_wide(a.c0.v, b.c0.v, T0);
  fmul_wide(a.c1.v, b.c1.v, T1);
  fmul_wide(sa, sb, T2);
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) T2[i] = subb32(T2[i], T0[i], br);
  br = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) T2[i] = subb32(T2[i], T1[i], br);
  br = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) T0[i] = subb32(T0[i], T1[i], br);
  const uint32_t mask = 0u - br;
  c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) T0[8 + i] = addc32(T0[8 + i], FpParams::MOD[i] & mask, c);
  return {fred_wide<FpParams>(T0), fred_wide<FpParams>(T2)};
#else
  Fp t0 = fmul(a.c0, b.c0);
  Fp t1 = fmul(a.c1, b.c1);
  Fp t2 = fmul(fadd(a.c0, a.c1), fadd(b.c0, b.c1));
  return {fsub(t0, t1), fsub(fsub(t2, t0), t1)};
#endif
}
DX_HD Fp2 sqr(const Fp2 &a) {
  Fp t = fmul(a.c0, a.c1);
  return {fmul(fadd(a.c0, a.c1), fsub(a.c0, a.c1)), fdbl(t)};
}
DX_HD Fp2 mul_fp(const Fp2 &a, const Fp &b) { return {fmul(a.c0, b), fmul(a.c1, b)}; }
// * xi = (9 + i)
DX_HD Fp2 mul_xi(const Fp2 &a) {
  Fp a0x8 = fdbl(fdbl(fdbl(a.c0)));
  Fp a1x8 = fdbl(fdbl(fdbl(a.c1)));
  return {fsub(fadd(a0x8, a.c0), a.c1), fadd(fadd(a1x8, a.c1), a.c0)};
}
DX_NI Fp2 inv(const Fp2 &a) {
  Fp t = finv(fadd(fsqr(a.c0), fsqr(a.c1)));
  return {fmul(a.c0, t), fneg(fmul(a.c1, t))};
}

struct Fp6 {
  Fp2 c0, c1, c2;
  static DX_HD Fp6 zero() { return {Fp2::zero(), Fp2::zero(), Fp2::zero()}; }
  static DX_HD Fp6 one() { return {Fp2::one(), Fp2::zero(), Fp2::zero()}; }
  DX_HD bool operator==(const Fp6 &o) const { return c0 == o.c0 && c1 == o.c1 && c2 == o.c2; }
};

DX_HD Fp6 add(const Fp6 &a, const Fp6 &b) { return {add(a.c0, b.c0), add(a.c1, b.c1), add(a.c2, b.c2)}; }
DX_HD Fp6 sub(const Fp6 &a, const Fp6 &b) { return {sub(a.c0, b.c0), sub(a.c1, b.c1), sub(a.c2, b.c2)}; }
DX_HD Fp6 neg(const Fp6 &a) { return {neg(a.c0), neg(a.c1), neg(a.c2)}; }
// Karatsuba-style 6-multiplication Fp6 product.
DX_NI Fp6 mul(const Fp6 &a, const Fp6 &b) {
  Fp2 t0 = mul(a.c0, b.c0), t1 = mul(a.c1, b.c1), t2 = mul(a.c2, b.c2);
  Fp2 c0 = add(t0, mul_xi(sub(sub(mul(add(a.c1, a.c2), add(b.c1, b.c2)), t1), t2)));
  Fp2 c1 = add(sub(sub(mul(add(a.c0, a.c1), add(b.c0, b.c1)), t0), t1), mul_xi(t2));
  Fp2 c2 = add(sub(sub(mul(add(a.c0, a.c2), add(b.c0, b.c2)), t0), t2), t1);
  return {c0, c1, c2};
}
DX_NI Fp6 sqr(const Fp6 &a) {
  // CH-SQR2
  Fp2 s0 = sqr(a.c0);
  Fp2 ab = mul(a.c0, a.c1);
  Fp2 s1 = dbl(ab);
  Fp2 s2 = sqr(add(sub(a.c0, a.c1), a.c2));
  Fp2 bc = mul(a.c1, a.c2);
  Fp2 s3 = dbl(bc);
  Fp2 s4 = sqr(a.c2);
  return {add(s0, mul_xi(s3)), add(s1, mul_xi(s4)), sub(sub(add(add(s1, s2), s3), s0), s4)};
}
DX_HD Fp6 mul_v(const Fp6 &a) { return {mul_xi(a.c2), a.c0, a.c1}; }
DX_HD Fp6 mul_fp2(const Fp6 &a, const Fp2 &b) { return {mul(a.c0, b), mul(a.c1, b), mul(a.c2, b)}; }
DX_NI Fp6 inv(const Fp6 &a) {
  Fp2 A = sub(sqr(a.c0), mul_xi(mul(a.c1, a.c2)));
  Fp2 B = sub(mul_xi(sqr(a.c2)), mul(a.c0, a.c1));
  Fp2 C = sub(sqr(a.c1), mul(a.c0, a.c2));
  Fp2 F = add(mul(a.c0, A), mul_xi(add(mul(a.c2, B), mul(a.c1, C))));
  Fp2 Fi = inv(F);
  return {mul(A, Fi), mul(B, Fi), mul(C, Fi)};
}

struct Fp12 {
  Fp6 c0, c1;
  static DX_HD Fp12 one() { return {Fp6::one(), Fp6::zero()}; }
  DX_HD bool operator==(const Fp12 &o) const { return c0 == o.c0 && c1 == o.c1; }
  DX_HD bool is_one() const { return *this == one(); }
};

DX_NI Fp12 mul(const Fp12 &a, const Fp12 &b) {
  Fp6 t0 = mul(a.c0, b.c0), t1 = mul(a.c1, b.c1);
  Fp6 c1 = sub(sub(mul(add(a.c0, a.c1), add(b.c0, b.c1)), t0), t1);
  return {add(t0, mul_v(t1)), c1};
}
DX_NI Fp12 sqr(const Fp12 &a) {
  // complex squaring: (a0 + a1 w)^2 = (a0+a1)(a0+v a1) - t - v t + 2 t w, t = a0 a1
  Fp6 t = mul(a.c0, a.c1);
  Fp6 c0 = sub(sub(mul(add(a.c0, a.c1), add(a.c0, mul_v(a.c1))), t), mul_v(t));
  return {c0, add(t, t)};
}
DX_HD Fp12 conj(const Fp12 &a) { return {a.c0, neg(a.c1)}; }
DX_NI Fp12 inv(const Fp12 &a) {
  Fp6 t = inv(sub(sqr(a.c0), mul_v(sqr(a.c1))));
  return {mul(a.c0, t), neg(mul(a.c1, t))};
}

// Sparse product f * (l0 + l1 w + l3 w^3): line values of the Miller loop
// (c0 = (l0,0,0), c1 = (l1,l3,0)).  13 Fp2 muls instead of 18.
DX_NI Fp12 mul_line(const Fp12 &f, const Fp2 &l0, const Fp2 &l1, const Fp2 &l3) {
  // a = f.c0, b = f.c1 ; L0 = (l0,0,0), L1 = (l1,l3,0)
  Fp6 t0 = mul_fp2(f.c0, l0);
  // t1 = f.c1 * (l1 + l3 v)
  const Fp6 &b = f.c1;
  Fp2 u0 = mul(b.c0, l1), u1 = mul(b.c1, l3);
  Fp6 t1 = {add(u0, mul_xi(mul(b.c2, l3))),
            sub(sub(mul(add(b.c0, b.c1), add(l1, l3)), u0), u1),
            add(mul(b.c2, l1), u1)};
  // (f.c0 + f.c1) * (l0 + l1 + l3 v)
  Fp6 s = add(f.c0, f.c1);
  Fp2 m0 = add(l0, l1);
  Fp2 v0 = mul(s.c0, m0), v1 = mul(s.c1, l3);
  Fp6 t2 = {add(v0, mul_xi(mul(s.c2, l3))),
            sub(sub(mul(add(s.c0, s.c1), add(m0, l3)), v0), v1),
            add(mul(s.c2, m0), v1)};
  return {add(t0, mul_v(t1)), sub(sub(t2, t0), t1)};
}

// Frobenius x -> x^(p^k), k in {1,2,3}: coefficient of w^e gets gamma_k[e]
// (and conjugation for odd k).
template <int K>
DX_NI Fp12 frob(const Fp12 &x) {
  const uint32_t(*G)[2][8] = (K == 1) ? Frob::G1 : (K == 2 ? Frob::G2 : Frob::G3);
  auto f = [&](const Fp2 &a, int e) {
    Fp2 aa = (K & 1) ? conj(a) : a;
    return mul(aa, Fp2::from_limbs(G[e]));
  };
  // tower index -> w exponent: c0.cj -> 2j ; c1.cj -> 2j+1
  return {{f(x.c0.c0, 0), f(x.c0.c1, 2), f(x.c0.c2, 4)}, {f(x.c1.c0, 1), f(x.c1.c1, 3), f(x.c1.c2, 5)}};
}

// Granger–Scott squaring for elements of the cyclotomic subgroup
// (valid after the easy part of the final exponentiation).
DX_HD void fp4_sqr(Fp2 &r0, Fp2 &r1, const Fp2 &a, const Fp2 &b) {
  Fp2 t0 = sqr(a), t1 = sqr(b);
  r0 = add(mul_xi(t1), t0);
  r1 = sub(sub(sqr(add(a, b)), t0), t1);
}
DX_NI Fp12 cyclotomic_sqr(const Fp12 &x) {
  // View Fp12 = Fp4[w]/(w^3 - z), Fp4 = Fp2[z]/(z^2 - xi), z = w^3, and
  // x = A + B w + C w^2 with A = g0 + g3 z, B = g1 + g4 z, C = g2 + g5 z
  // (g_e = coefficient of w^e: g0=c0.c0 g2=c0.c1 g4=c0.c2 g1=c1.c0 g3=c1.c1 g5=c1.c2).
  // x^2 = (3A^2 - 2conj A) + (3 z C^2 + 2 conj B) w + (3B^2 - 2 conj C) w^2.
  const Fp2 &g0 = x.c0.c0, &g2 = x.c0.c1, &g4 = x.c0.c2;
  const Fp2 &g1 = x.c1.c0, &g3 = x.c1.c1, &g5 = x.c1.c2;
  Fp2 A0, A1, B0, B1, C0, C1;
  fp4_sqr(A0, A1, g0, g3);
  fp4_sqr(B0, B1, g1, g4);
  fp4_sqr(C0, C1, g2, g5);
  Fp12 r;
  r.c0.c0 = add(dbl(sub(A0, g0)), A0);  // h0 = 3A0 - 2g0
  r.c1.c1 = add(dbl(add(A1, g3)), A1);  // h3 = 3A1 + 2g3
  Fp2 xc1 = mul_xi(C1);
  r.c1.c0 = add(dbl(add(xc1, g1)), xc1);  // h1 = 3 xi C1 + 2g1
  r.c0.c2 = add(dbl(sub(C0, g4)), C0);    // h4 = 3C0 - 2g4
  r.c0.c1 = add(dbl(sub(B0, g2)), B0);    // h2 = 3B0 - 2g2
  r.c1.c2 = add(dbl(add(B1, g5)), B1);    // h5 = 3B1 + 2g5
  return r;
}

// x^u for the BN parameter u (x in the cyclotomic subgroup).
DX_NI Fp12 cyc_pow_u(const Fp12 &x) {
  Fp12 r = x;
  for (int b = 61; b >= 0; b--) {  // u has bit 62 as MSB
    r = cyclotomic_sqr(r);
    if ((BN_U >> b) & 1ull) r = mul(r, x);
  }
  return r;
}

// Exact final exponentiation f^((p^12-1)/r) — same chain as
// oracle.final_exp_fast (Scott et al. hard part).
DX_NI Fp12 final_exp(const Fp12 &f) {
  Fp12 t = mul(conj(f), inv(f));
  t = mul(frob<2>(t), t);
  Fp12 fu = cyc_pow_u(t);
  Fp12 fu2 = cyc_pow_u(fu);
  Fp12 fu3 = cyc_pow_u(fu2);
  Fp12 y3 = conj(frob<1>(fu));
  Fp12 fu2p = frob<1>(fu2);
  Fp12 fu3p = frob<1>(fu3);
  Fp12 y2 = frob<2>(fu2);
  Fp12 y0 = mul(mul(frob<1>(t), frob<2>(t)), frob<3>(t));
  Fp12 y1 = conj(t);
  Fp12 y5 = conj(fu2);
  Fp12 y4 = conj(mul(fu, fu2p));
  Fp12 y6 = conj(mul(fu3, fu3p));
  Fp12 t0 = mul(mul(cyclotomic_sqr(y6), y4), y5);
  Fp12 t1 = mul(mul(y3, y5), t0);
  t0 = mul(t0, y2);
  t1 = mul(cyclotomic_sqr(t1), t0);
  t1 = cyclotomic_sqr(t1);
  t0 = mul(t1, y1);
  t1 = mul(t1, y0);
  t0 = mul(cyclotomic_sqr(t0), t1);
  return t0;
}

}  // namespace dx
