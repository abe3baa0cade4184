// GLV decomposition of a full 256-bit G1 scalar: k = k1 + k2 * lambda (mod r)
// with 0 <= k1 < 2^128 and |k2| < 2^128, so a variable-base multiplication
// k P = k1 P + k2 phi(P) runs a 128-step ladder over (P, phi(P)) instead of a
// 256-step one (phi(x, y) = (beta x, y), lambda = native.GLV_LAMBDA).
//
// Babai rounding (floor form) against the reduced basis of
// {(a, b) : a + b lambda = 0 mod r}:
//   v1 = (A1, -B1), v2 = (A2, B2),  A1 = B2 = 0x89d3256894d213e3,
//   A2 = 0x6f4d8248eeb859fd0be4e1541221250b, B1 = 0x6f4d8248eeb859fc8211bbeb7d4f1128
// c1 = floor(k G1 / 2^256), c2 = floor(k G2 / 2^256) with G1 = floor(B2 2^256 / r),
// G2 = floor(B1 2^256 / r); k1 = k - c1 A1 - c2 A2, k2 = c1 B1 - c2 B2.
// The residual (k1, k2) = d1 v1 + d2 v2 with d1, d2 in [0, 2) (one unit from
// the floor, < 1 from truncating G), hence the bounds above for EVERY k < 2^256
// (checked over 3e5 random and edge scalars by tools' derivation and by
// tests/test_glv_split.py against Python integers).
#pragma once
#include <stdint.h>

#include "field.h"

namespace dx {

namespace glv {
struct C {  // little-endian 32-bit words
  static constexpr uint32_t G1w[3] = {0xc7e0b3d7u, 0xd91d232eu, 0x2u};
  static constexpr uint32_t G2w[5] = {0x391eb18du, 0x7a7bd9d4u, 0xa773d2cfu, 0x4ccef014u, 0x2u};
  static constexpr uint32_t A1w[2] = {0x94d213e3u, 0x89d32568u};
  static constexpr uint32_t A2w[4] = {0x1221250bu, 0x0be4e154u, 0xeeb859fdu, 0x6f4d8248u};
  static constexpr uint32_t B1w[4] = {0x7d4f1128u, 0x8211bbebu, 0xeeb859fcu, 0x6f4d8248u};
};

// high words (index >= 8) of k[8] * g[NG] -> c[NG + 1] (the true value fits: c < 2^160)
template <int NG>
DX_HD void mul_hi(const uint32_t *k, const uint32_t *g, uint32_t *c) {
  uint32_t t[8 + NG + 1];
#pragma unroll
  for (int i = 0; i < 8 + NG + 1; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < NG; j++) {
      const uint64_t s = (uint64_t)k[i] * g[j] + t[i + j] + carry;
      t[i + j] = (uint32_t)s;
      carry = s >> 32;
    }
    t[i + NG] = (uint32_t)carry;
  }
#pragma unroll
  for (int i = 0; i <= NG; i++) c[i] = t[i + 8];
}

// acc[N] -= a[NA] * b[NB]  (mod 2^(32 N))
template <int N, int NA, int NB>
DX_HD void sub_mul(uint32_t *acc, const uint32_t *a, const uint32_t *b) {
  uint32_t p[N];
#pragma unroll
  for (int i = 0; i < N; i++) p[i] = 0;
#pragma unroll
  for (int i = 0; i < NA; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < NB; j++) {
      if (i + j >= N) break;
      const uint64_t s = (uint64_t)a[i] * b[j] + p[i + j] + carry;
      p[i + j] = (uint32_t)s;
      carry = s >> 32;
    }
    if (i + NB < N) p[i + NB] += (uint32_t)carry;
  }
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    const uint64_t d = (uint64_t)acc[i] - p[i] - borrow;
    acc[i] = (uint32_t)d;
    borrow = (d >> 63) & 1u;
  }
}
}  // namespace glv

// k[8] (any value < 2^256) -> k1[4] (>= 0), k2[4] = |k2|, neg2 = (k2 < 0)
DX_HD void glv_split(const uint32_t *k, uint32_t *k1, uint32_t *k2, bool &neg2) {
  uint32_t c1[4], c2[6];
  glv::mul_hi<3>(k, glv::C::G1w, c1);
  glv::mul_hi<5>(k, glv::C::G2w, c2);
  // k1 = k - c1 A1 - c2 A2 (mod 2^128; the true value is in [0, 2^128))
  uint32_t a[4] = {k[0], k[1], k[2], k[3]};
  glv::sub_mul<4, 4, 2>(a, c1, glv::C::A1w);
  glv::sub_mul<4, 5, 4>(a, c2, glv::C::A2w);
  // k2 = c1 B1 - c2 B2 (mod 2^160; |true value| < 2^128)
  uint32_t b[5] = {0, 0, 0, 0, 0};
  glv::sub_mul<5, 5, 2>(b, c2, glv::C::A1w);  // B2 == A1
  uint32_t nb[5] = {0, 0, 0, 0, 0};
  glv::sub_mul<5, 4, 4>(nb, c1, glv::C::B1w);  // nb = -c1 B1
  // b = -c2 B2 - (-c1 B1)
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const uint64_t d = (uint64_t)b[i] - nb[i] - borrow;
    b[i] = (uint32_t)d;
    borrow = (d >> 63) & 1u;
  }
  neg2 = (b[4] >> 31) != 0;
  if (neg2) {  // magnitude
    uint64_t c = 1;
#pragma unroll
    for (int i = 0; i < 5; i++) {
      const uint64_t s = (uint64_t)(~b[i]) + c;
      b[i] = (uint32_t)s;
      c = s >> 32;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    k1[i] = a[i];
    k2[i] = b[i];
  }
}

}  // namespace dx
