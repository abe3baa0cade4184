// Optimal-ate pairing on BN254: projective Miller loop over the NAF of 6u+2
// with sparse line multiplication, then the exact final exponentiation.
// Replaces kyber bn256 `Pair` (external), called by the reference at
// lib/range/range_proof.go:396-397 (prove) and :540-544 (verify).
// Algorithm validated step-for-step against drynx_amd/crypto/oracle.py.
#pragma once
#include "curve.h"

namespace dx {

struct LineCoeffs {
  Fp2 l0, l1, l3;
};

// Doubling step, homogeneous projective T = (X:Y:Z) on the twist, x = X/Z.
DX_NI void miller_dbl(Fp2 &X, Fp2 &Y, Fp2 &Z, const Fp &xP, const Fp &yP, LineCoeffs &l) {
  const Fp2 b2 = Fp2::from_limbs(Curve::B2);
  Fp2 A = mul(X, Y);                 // XY  (halving folded below)
  Fp2 Bq = sqr(Y);
  Fp2 C = sqr(Z);
  Fp2 E = mul(add(dbl(C), C), b2);   // 3 b' Z^2
  Fp2 F = add(dbl(E), E);            // 3E
  Fp2 H = sub(sub(sqr(add(Y, Z)), Bq), C);  // 2YZ
  // X3 = XY/2 (B - F) ; Y3 = ((B+F)/2)^2 - 3E^2 ; Z3 = B H
  // Scale the whole point by 4 (projective, allowed): X3' = 2XY(B-F), Y3' = (B+F)^2 - 12E^2, Z3' = 4BH
  Fp2 X3 = dbl(mul(A, sub(Bq, F)));
  Fp2 E2 = sqr(E);
  Fp2 Y3 = sub(sqr(add(Bq, F)), dbl(dbl(add(dbl(E2), E2))));
  Fp2 Z3 = dbl(dbl(mul(Bq, H)));
  l.l0 = neg(mul_fp(H, yP));
  Fp2 X2 = sqr(X);
  l.l1 = mul_fp(add(dbl(X2), X2), xP);
  l.l3 = sub(E, Bq);
  X = X3; Y = Y3; Z = Z3;
}

// Mixed addition step T + Q (Q affine on the twist).
DX_NI void miller_add(Fp2 &X, Fp2 &Y, Fp2 &Z, const Fp2 &x2, const Fp2 &y2, const Fp &xP, const Fp &yP,
                      LineCoeffs &l) {
  Fp2 th = sub(Y, mul(y2, Z));
  Fp2 la = sub(X, mul(x2, Z));
  Fp2 C = sqr(th), D = sqr(la);
  Fp2 E = mul(D, la), F = mul(Z, C), G = mul(X, D);
  Fp2 H = sub(add(E, F), dbl(G));
  Fp2 X3 = mul(la, H);
  Fp2 Y3 = sub(mul(th, sub(G, H)), mul(Y, E));
  Fp2 Z3 = mul(Z, E);
  l.l0 = mul_fp(la, yP);
  l.l1 = neg(mul_fp(th, xP));
  l.l3 = sub(mul(th, x2), mul(la, y2));
  X = X3; Y = Y3; Z = Z3;
}

// Miller loop f_{6u+2,Q}(P) * l_{T,pi(Q)} * l_{T',-pi^2(Q)} (not final-exponentiated).
DX_NI Fp12 miller_loop(const G1A &P, const G2A &Q) {
  if (P.is_inf() || Q.is_inf()) return Fp12::one();
  const Fp &xP = P.x, &yP = P.y;
  Fp2 X = Q.x, Y = Q.y, Z = Fp2::one();
  Fp2 nQy = neg(Q.y);
  Fp12 f = Fp12::one();
  LineCoeffs l;
  for (int i = ATE_NAF_LEN - 2; i >= 0; i--) {
    miller_dbl(X, Y, Z, xP, yP, l);
    f = mul_line(sqr(f), l.l0, l.l1, l.l3);
    int d = ATE_NAF[i];
    if (d != 0) {
      miller_add(X, Y, Z, Q.x, d > 0 ? Q.y : nQy, xP, yP, l);
      f = mul_line(f, l.l0, l.l1, l.l3);
    }
  }
  Fp2 q1x = mul(conj(Q.x), Fp2::from_limbs(Frob::TWX1));
  Fp2 q1y = mul(conj(Q.y), Fp2::from_limbs(Frob::TWY1));
  Fp2 q2x = mul(Q.x, Fp2::from_limbs(Frob::TWX2));
  Fp2 q2y = neg(mul(Q.y, Fp2::from_limbs(Frob::TWY2)));
  miller_add(X, Y, Z, q1x, q1y, xP, yP, l);
  f = mul_line(f, l.l0, l.l1, l.l3);
  miller_add(X, Y, Z, q2x, q2y, xP, yP, l);
  f = mul_line(f, l.l0, l.l1, l.l3);
  return f;
}

DX_NI Fp12 pairing(const G1A &P, const G2A &Q) { return final_exp(miller_loop(P, Q)); }

// GT exponentiation by a 256-bit scalar (cyclotomic squarings).
DX_NI Fp12 gt_pow(const Fp12 &x, const uint32_t *k) {
  Fp12 r = Fp12::one();
  int top = 255;
  while (top > 0 && ((k[top >> 5] >> (top & 31)) & 1u) == 0) top--;
  for (int i = top; i >= 0; i--) {
    r = cyclotomic_sqr(r);
    if ((k[i >> 5] >> (i & 31)) & 1u) r = mul(r, x);
  }
  return r;
}

// Fixed-base GT exponentiation with a comb table: table[w*256+d] = base^(d*2^(8w)).
DX_NI Fp12 gt_fixed_pow(const Fp12 *table, const uint32_t *k) {
  Fp12 r = Fp12::one();
  for (int w = 0; w < 32; w++) {
    uint32_t d = (k[w >> 2] >> ((w & 3) * 8)) & 255u;
    if (d) r = mul(r, table[w * 256 + d]);
  }
  return r;
}

// 4-bit comb: table[w*15 + d - 1] = base^(d * 16^w), w < 64 (360 KiB per base).
DX_NI Fp12 gt_fixed_pow4(const Fp12 *table, const uint32_t *k) {
  Fp12 r = Fp12::one();
  for (int w = 0; w < 64; w++) {
    uint32_t d = (k[w >> 3] >> ((w & 7) * 4)) & 15u;
    if (d) r = mul(r, table[w * 15 + d - 1]);
  }
  return r;
}

}  // namespace dx
