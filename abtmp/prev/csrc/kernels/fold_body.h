// Two-phase batched Miller fold of the range-proof verifier (K16 hot loop),
// included by dx_fold.hip (tower functions out of line) and dx_fold_inl.hip
// (everything force-inlined); FOLD_SFX names the variant's entry points.
//
// The verifier needs prod_it ML(P_it, V_it) over ~1e6 items per VN inbox
// (lib/range/range_proof.go:522-553 computes 3 pairings per item instead).
// One fused kernel per item holds the Fp12 accumulator (96 VGPRs), the twist
// point (48), the G2 operand (32) and the tower temporaries at once, which
// capped it at 256 VGPRs with call-frame spills.  Here:
//   phase 1 (rp_lines): per item, the G2 side of the Miller loop only -- the
//     88 sparse line values (l0, l1, l3) evaluated at P, streamed to HBM in a
//     coalesced [step][12][item] uint4 image (192 B per step and item);
//   phase 2 (rp_accum): per lane K items share ONE accumulator,
//     f <- f^2 * prod_k l_k(P_k) (a multi-Miller loop: one Fp12 squaring per
//     step for K items instead of K), then the LDS tree folds the workgroup.
// The product over items is all the batch equation needs.
#pragma once
#include "common.h"
#include "../bn254/g1_fast.h"

// Occupancy target of the line and accumulation kernels (a variant TU may ask
// for 1 wave per SIMD: 512 registers, AGPRs as spill space instead of scratch).
#ifndef FOLD_OCC
#define FOLD_OCC DX_OCC
#endif

#define FOLD_CAT2(a, b) a##b
#define FOLD_CAT(a, b) FOLD_CAT2(a, b)
#define FOLD_NAME(x) FOLD_CAT(x, FOLD_SFX)

namespace FOLD_NAME(fold_ns_) {

constexpr int kWG = 64;
constexpr int count_add_steps() {
  int c = 0;
  for (int i = ATE_NAF_LEN - 2; i >= 0; i--) c += ATE_NAF[i] != 0 ? 1 : 0;
  return c;
}
constexpr int kSteps = (ATE_NAF_LEN - 1) + count_add_steps() + 2;  // doublings + NAF additions + 2 Frobenius lines

// line image: uint4 word q (0..11) of step s, item it at lines[(s*12 + q)*n + it]
__device__ __forceinline__ void store_line(uint4 *lines, int64_t n, int s, int64_t it, const Fp2 &l0, const Fp2 &l1,
                                           const Fp2 &l3) {
  const Fp2 *src[3] = {&l0, &l1, &l3};
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(src[c]);
#pragma unroll
    for (int q = 0; q < 4; q++)
      lines[((int64_t)s * 12 + c * 4 + q) * n + it] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
  }
}

__device__ __forceinline__ void load_line(const uint4 *__restrict__ lines, int64_t n, int s, int64_t it, Fp2 &l0,
                                          Fp2 &l1, Fp2 &l3) {
  Fp2 *dst[3] = {&l0, &l1, &l3};
#pragma unroll
  for (int c = 0; c < 3; c++) {
    uint32_t *w = reinterpret_cast<uint32_t *>(dst[c]);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint4 v = lines[((int64_t)s * 12 + c * 4 + q) * n + it];
      w[4 * q] = v.x;
      w[4 * q + 1] = v.y;
      w[4 * q + 2] = v.z;
      w[4 * q + 3] = v.w;
    }
  }
}

// Same formulas as pairing.h miller_dbl / miller_add (validated against the
// oracle), reordered so each line value is stored as soon as it exists and
// the twist-point update runs with the line temporaries already dead.
__device__ __forceinline__ void line_dbl(Fp2 &X, Fp2 &Y, Fp2 &Z, const Fp &xP, const Fp &yP, uint4 *lines, int64_t n,
                                         int s, int64_t it) {
  const Fp2 b2 = Fp2::from_limbs(Curve::B2);
  Fp2 X2 = sqr(X);
  const Fp2 l1 = mul_fp(add(dbl(X2), X2), xP);
  Fp2 Bq = sqr(Y);
  Fp2 C = sqr(Z);
  Fp2 H = sub(sub(sqr(add(Y, Z)), Bq), C);
  const Fp2 l0 = neg(mul_fp(H, yP));
  Fp2 E = mul(add(dbl(C), C), b2);
  const Fp2 l3 = sub(E, Bq);
  store_line(lines, n, s, it, l0, l1, l3);
  Fp2 F = add(dbl(E), E);
  Fp2 A = mul(X, Y);
  X = dbl(mul(A, sub(Bq, F)));
  Z = dbl(dbl(mul(Bq, H)));
  Fp2 E2 = sqr(E);
  Y = sub(sqr(add(Bq, F)), dbl(dbl(add(dbl(E2), E2))));
}

__device__ __forceinline__ void line_add(Fp2 &X, Fp2 &Y, Fp2 &Z, const Fp2 &x2, const Fp2 &y2, const Fp &xP,
                                         const Fp &yP, uint4 *lines, int64_t n, int s, int64_t it) {
  Fp2 th = sub(Y, mul(y2, Z));
  Fp2 la = sub(X, mul(x2, Z));
  store_line(lines, n, s, it, mul_fp(la, yP), neg(mul_fp(th, xP)), sub(mul(th, x2), mul(la, y2)));
  Fp2 C = sqr(th), D = sqr(la);
  Fp2 E = mul(D, la), F = mul(Z, C), G = mul(X, D);
  Fp2 H = sub(add(E, F), dbl(G));
  Y = sub(mul(th, sub(G, H)), mul(Y, E));
  X = mul(la, H);
  Z = mul(Z, E);
}

// Items it < n; several verifiers' batches over the same V may share one
// launch: item it pairs P[it] with V[it % period] (period = n for one batch;
// rows of P past a batch's own length are the point at infinity).
__global__ void __launch_bounds__(kWG) FOLD_OCC rp_lines_kernel(const uint32_t *__restrict__ P_aff,
                                                              const uint32_t *__restrict__ V_aff,
                                                              uint4 *__restrict__ lines, int64_t n,
                                                              int64_t period, int64_t n_v) {
  const int64_t it = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (it >= n) return;
  const int64_t q = it % period;
  const G1A P = at<G1A>(P_aff, it);
  const G2A Q = at<G2A>(V_aff, q < n_v ? q : 0);
  if (P.is_inf() || Q.is_inf()) {  // ML = 1: identity lines
    for (int s = 0; s < kSteps; s++) store_line(lines, n, s, it, Fp2::one(), Fp2::zero(), Fp2::zero());
    return;
  }
  Fp2 X = Q.x, Y = Q.y, Z = Fp2::one();
  int s = 0;
  for (int i = ATE_NAF_LEN - 2; i >= 0; i--) {
    line_dbl(X, Y, Z, P.x, P.y, lines, n, s++, it);
    const int d = ATE_NAF[i];
    if (d != 0) {
      // re-read Q at each addition step instead of pinning 32 VGPRs for it
      asm volatile("" ::: "memory");
      const G2A qq = at<G2A>(V_aff, q < n_v ? q : 0);
      line_add(X, Y, Z, qq.x, d > 0 ? qq.y : neg(qq.y), P.x, P.y, lines, n, s++, it);
    }
  }
  asm volatile("" ::: "memory");
  const G2A qq = at<G2A>(V_aff, q < n_v ? q : 0);
  line_add(X, Y, Z, mul(conj(qq.x), Fp2::from_limbs(Frob::TWX1)), mul(conj(qq.y), Fp2::from_limbs(Frob::TWY1)), P.x,
           P.y, lines, n, s++, it);
  line_add(X, Y, Z, mul(qq.x, Fp2::from_limbs(Frob::TWX2)), neg(mul(qq.y, Fp2::from_limbs(Frob::TWY2))), P.x, P.y,
           lines, n, s++, it);
}

// ---- shared-V variant: the line COEFFICIENTS depend on V only (the
// evaluation at P is two Fp2-by-Fp products), so verifiers folding the same
// proofs with their own weights share one coefficient image:
//   l0 = c0 * yP, l1 = c1 * xP, l3 = c3
// (dbl: c0 = -H, c1 = 3X^2, c3 = E - B; add: c0 = lambda, c1 = -theta,
// c3 = theta x2 - lambda y2).  The accumulation evaluates at P as it goes.
__device__ __forceinline__ void coef_dbl(Fp2 &X, Fp2 &Y, Fp2 &Z, uint4 *lines, int64_t n, int s, int64_t it) {
  const Fp2 b2 = Fp2::from_limbs(Curve::B2);
  Fp2 X2 = sqr(X);
  const Fp2 c1 = add(dbl(X2), X2);
  Fp2 Bq = sqr(Y);
  Fp2 C = sqr(Z);
  Fp2 H = sub(sub(sqr(add(Y, Z)), Bq), C);
  Fp2 E = mul(add(dbl(C), C), b2);
  store_line(lines, n, s, it, neg(H), c1, sub(E, Bq));
  Fp2 F = add(dbl(E), E);
  Fp2 A = mul(X, Y);
  X = dbl(mul(A, sub(Bq, F)));
  Z = dbl(dbl(mul(Bq, H)));
  Fp2 E2 = sqr(E);
  Y = sub(sqr(add(Bq, F)), dbl(dbl(add(dbl(E2), E2))));
}

__device__ __forceinline__ void coef_add(Fp2 &X, Fp2 &Y, Fp2 &Z, const Fp2 &x2, const Fp2 &y2, uint4 *lines,
                                         int64_t n, int s, int64_t it) {
  Fp2 th = sub(Y, mul(y2, Z));
  Fp2 la = sub(X, mul(x2, Z));
  store_line(lines, n, s, it, la, neg(th), sub(mul(th, x2), mul(la, y2)));
  Fp2 C = sqr(th), D = sqr(la);
  Fp2 E = mul(D, la), F = mul(Z, C), G = mul(X, D);
  Fp2 H = sub(add(E, F), dbl(G));
  Y = sub(mul(th, sub(G, H)), mul(Y, E));
  X = mul(la, H);
  Z = mul(Z, E);
}

// One item per V (m items); V at infinity gets zero coefficients (the
// accumulation skips it: ML(P, O) = 1).
__global__ void __launch_bounds__(kWG) FOLD_OCC rp_coeffs_kernel(const uint32_t *__restrict__ V_aff,
                                                               uint4 *__restrict__ lines, int64_t m) {
  const int64_t it = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (it >= m) return;
  const G2A Q = at<G2A>(V_aff, it);
  if (Q.is_inf()) {
    for (int s = 0; s < kSteps; s++) store_line(lines, m, s, it, Fp2::zero(), Fp2::zero(), Fp2::zero());
    return;
  }
  Fp2 X = Q.x, Y = Q.y, Z = Fp2::one();
  int s = 0;
  for (int i = ATE_NAF_LEN - 2; i >= 0; i--) {
    coef_dbl(X, Y, Z, lines, m, s++, it);
    const int d = ATE_NAF[i];
    if (d != 0) {
      asm volatile("" ::: "memory");
      const G2A qq = at<G2A>(V_aff, it);
      coef_add(X, Y, Z, qq.x, d > 0 ? qq.y : neg(qq.y), lines, m, s++, it);
    }
  }
  asm volatile("" ::: "memory");
  const G2A qq = at<G2A>(V_aff, it);
  coef_add(X, Y, Z, mul(conj(qq.x), Fp2::from_limbs(Frob::TWX1)), mul(conj(qq.y), Fp2::from_limbs(Frob::TWY1)),
           lines, m, s++, it);
  coef_add(X, Y, Z, mul(qq.x, Fp2::from_limbs(Frob::TWX2)), neg(mul(qq.y, Fp2::from_limbs(Frob::TWY2))), lines, m,
           s++, it);
}

template <int K>
__device__ __forceinline__ void accum_p_step(Fp12 &f, const uint4 *__restrict__ coef, const uint32_t *__restrict__ P_aff,
                                             int64_t m, int s, int64_t qbase, int64_t pbase, uint32_t live) {
#pragma unroll 1
  for (int k = 0; k < K; k++) {
    if ((live >> k) & 1u) {
      Fp2 c0, c1, c3;
      load_line(coef, m, s, qbase + (int64_t)k * kWG, c0, c1, c3);
      const G1A P = at<G1A>(P_aff, pbase + (int64_t)k * kWG);
      f = mul_line(f, mul_fp(c0, P.y), mul_fp(c1, P.x), c3);
    }
  }
}

// G verifiers' point images P[v * period + q] (q < m live) against ONE
// coefficient image.  Block b runs verifier v on coefficient block qb with
// the G blocks sharing qb dealt to one XCD back to back (blocks b and b + 8
// share an XCD), so the second and third reads of a coefficient come from
// that XCD's L2.  Requires period % (64 K 8) == 0.
template <int K>
__global__ void __launch_bounds__(kWG) FOLD_OCC rp_accum_p_kernel(const uint4 *__restrict__ coef,
                                                                const uint32_t *__restrict__ P_aff,
                                                                const uint32_t *__restrict__ V_aff, uint32_t *f_blk,
                                                                int64_t m, int64_t period, int G) {
  __shared__ Fp12 sf[kWG / 2];
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x, slot = b >> 3;
  const int v = (int)(slot % G);
  const int64_t qb = (slot / G) * 8 + (b & 7);
  const int64_t qbase = qb * kWG * K + lane, pbase = (int64_t)v * period + qbase;
  uint32_t live = 0;
#pragma unroll 1
  for (int k = 0; k < K; k++) {
    const int64_t q = qbase + (int64_t)k * kWG;
    if (q < m && !at<G1A>(P_aff, pbase + (int64_t)k * kWG).is_inf() && !at<G2A>(V_aff, q).is_inf()) live |= 1u << k;
  }
  Fp12 f = Fp12::one();
  int s = 0;
  for (int i = ATE_NAF_LEN - 2; i >= 0; i--) {
    if (i != ATE_NAF_LEN - 2) f = sqr(f);
    accum_p_step<K>(f, coef, P_aff, m, s++, qbase, pbase, live);
    if (ATE_NAF[i] != 0) accum_p_step<K>(f, coef, P_aff, m, s++, qbase, pbase, live);
  }
  accum_p_step<K>(f, coef, P_aff, m, s++, qbase, pbase, live);
  accum_p_step<K>(f, coef, P_aff, m, s++, qbase, pbase, live);
  for (int h = kWG / 2; h > 0; h >>= 1) {
    if (lane >= h && lane < 2 * h) sf[lane - h] = f;
    __syncthreads();
    if (lane < h) f = mul(f, sf[lane]);
    __syncthreads();
  }
  if (lane == 0) at<Fp12>(f_blk, (int64_t)v * (period / ((int64_t)kWG * K)) + qb) = f;
}

// ---- normalised shared-V variant (fold mode 4).  The final exponentiation
// kills every factor from Fp6 (p^6 - 1 divides (p^12 - 1) / r), so a line
// l0 + l1 w + l3 w^3 = (c0 yP) (1 + (c1/c0)(xP/yP) w + (c3/c0)(1/yP) w^3)
// may be replaced by 1 + (a u) w + (b v) w^3 with a = c1/c0, b = c3/c0 per V
// (normalised once, shared by every verifier: one Fp2 inversion per item via
// Montgomery's trick over its 88 steps) and u = xP/yP, v = 1/yP per point (the
// point kernel's one inversion).  The product by such a line costs 10 Fp2
// products instead of 13, and the image is 128 B per step instead of 192.
__device__ __forceinline__ void store_ab(uint4 *img, int64_t n, int s, int64_t it, const Fp2 &a, const Fp2 &b) {
  const Fp2 *src[2] = {&a, &b};
#pragma unroll
  for (int c = 0; c < 2; c++) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(src[c]);
#pragma unroll
    for (int q = 0; q < 4; q++)
      img[((int64_t)s * 8 + c * 4 + q) * n + it] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
  }
}

__device__ __forceinline__ void load_ab(const uint4 *__restrict__ img, int64_t n, int s, int64_t it, Fp2 &a, Fp2 &b) {
  Fp2 *dst[2] = {&a, &b};
#pragma unroll
  for (int c = 0; c < 2; c++) {
    uint32_t *w = reinterpret_cast<uint32_t *>(dst[c]);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint4 v = img[((int64_t)s * 8 + c * 4 + q) * n + it];
      w[4 * q] = v.x;
      w[4 * q + 1] = v.y;
      w[4 * q + 2] = v.z;
      w[4 * q + 3] = v.w;
    }
  }
}

// one Fp2 per step and item: scratch [step][4][n] uint4
__device__ __forceinline__ void store_fp2(uint4 *buf, int64_t n, int s, int64_t it, const Fp2 &x) {
  const uint32_t *w = reinterpret_cast<const uint32_t *>(&x);
#pragma unroll
  for (int q = 0; q < 4; q++) buf[((int64_t)s * 4 + q) * n + it] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

__device__ __forceinline__ Fp2 load_fp2(const uint4 *buf, int64_t n, int s, int64_t it) {
  Fp2 x;
  uint32_t *w = reinterpret_cast<uint32_t *>(&x);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint4 v = buf[((int64_t)s * 4 + q) * n + it];
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
  return x;
}

// forward half of a step: raw (c1, c3) to the image, c0 and the prefix product
// before it to scratch
__device__ __forceinline__ void ncoef_put(uint4 *img, uint4 *c0s, uint4 *pre, int64_t m, int s, int64_t it,
                                          const Fp2 &c0, const Fp2 &c1, const Fp2 &c3, Fp2 &prod) {
  store_ab(img, m, s, it, c1, c3);
  store_fp2(c0s, m, s, it, c0);
  store_fp2(pre, m, s, it, prod);
  prod = mul(prod, c0);
}

__global__ void __launch_bounds__(kWG) FOLD_OCC rp_ncoeffs_kernel(const uint32_t *__restrict__ V_aff,
                                                                uint4 *__restrict__ img, uint4 *__restrict__ c0s,
                                                                uint4 *__restrict__ pre, int64_t m) {
  const int64_t it = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (it >= m) return;
  const G2A Q = at<G2A>(V_aff, it);
  if (Q.is_inf()) {
    for (int s = 0; s < kSteps; s++) store_ab(img, m, s, it, Fp2::zero(), Fp2::zero());
    return;
  }
  const Fp2 b2 = Fp2::from_limbs(Curve::B2);
  Fp2 X = Q.x, Y = Q.y, Z = Fp2::one(), prod = Fp2::one();
  int s = 0;
  auto dbl_step = [&]() {
    Fp2 X2 = sqr(X);
    const Fp2 c1 = add(dbl(X2), X2);
    Fp2 Bq = sqr(Y);
    Fp2 C = sqr(Z);
    Fp2 H = sub(sub(sqr(add(Y, Z)), Bq), C);
    Fp2 E = mul(add(dbl(C), C), b2);
    ncoef_put(img, c0s, pre, m, s++, it, neg(H), c1, sub(E, Bq), prod);
    Fp2 F = add(dbl(E), E);
    Fp2 A = mul(X, Y);
    X = dbl(mul(A, sub(Bq, F)));
    Z = dbl(dbl(mul(Bq, H)));
    Fp2 E2 = sqr(E);
    Y = sub(sqr(add(Bq, F)), dbl(dbl(add(dbl(E2), E2))));
  };
  auto add_step = [&](const Fp2 &x2, const Fp2 &y2) {
    Fp2 th = sub(Y, mul(y2, Z));
    Fp2 la = sub(X, mul(x2, Z));
    ncoef_put(img, c0s, pre, m, s++, it, la, neg(th), sub(mul(th, x2), mul(la, y2)), prod);
    Fp2 C = sqr(th), D = sqr(la);
    Fp2 E = mul(D, la), F = mul(Z, C), G = mul(X, D);
    Fp2 H = sub(add(E, F), dbl(G));
    Y = sub(mul(th, sub(G, H)), mul(Y, E));
    X = mul(la, H);
    Z = mul(Z, E);
  };
  for (int i = ATE_NAF_LEN - 2; i >= 0; i--) {
    dbl_step();
    const int d = ATE_NAF[i];
    if (d != 0) {
      asm volatile("" ::: "memory");
      const G2A qq = at<G2A>(V_aff, it);
      add_step(qq.x, d > 0 ? qq.y : neg(qq.y));
    }
  }
  asm volatile("" ::: "memory");
  {
    const G2A qq = at<G2A>(V_aff, it);
    add_step(mul(conj(qq.x), Fp2::from_limbs(Frob::TWX1)), mul(conj(qq.y), Fp2::from_limbs(Frob::TWY1)));
  }
  asm volatile("" ::: "memory");
  {
    const G2A qq = at<G2A>(V_aff, it);
    add_step(mul(qq.x, Fp2::from_limbs(Frob::TWX2)), neg(mul(qq.y, Fp2::from_limbs(Frob::TWY2))));
  }
  // backward: (c1, c3) / c0 with one inversion (Montgomery's trick)
  Fp2 inv = ::dx::inv(prod);
  for (int t = kSteps - 1; t >= 0; t--) {
    const Fp2 inv_t = mul(inv, load_fp2(pre, m, t, it));
    inv = mul(inv, load_fp2(c0s, m, t, it));
    Fp2 a, b;
    load_ab(img, m, t, it, a, b);
    store_ab(img, m, t, it, mul(a, inv_t), mul(b, inv_t));
  }
}

// f * (1 + l1 w + l3 w^3): 10 Fp2 products
__device__ __forceinline__ Fp12 mul_line1(const Fp12 &f, const Fp2 &l1, const Fp2 &l3) {
  const Fp6 &g = f.c1;
  const Fp2 u0 = mul(g.c0, l1), u1 = mul(g.c1, l3);
  const Fp6 t1 = {add(u0, mul_xi(mul(g.c2, l3))), sub(sub(mul(add(g.c0, g.c1), add(l1, l3)), u0), u1),
                  add(mul(g.c2, l1), u1)};
  const Fp6 sm = add(f.c0, f.c1);
  const Fp2 m0 = add(Fp2::one(), l1);
  const Fp2 v0 = mul(sm.c0, m0), v1 = mul(sm.c1, l3);
  const Fp6 t2 = {add(v0, mul_xi(mul(sm.c2, l3))), sub(sub(mul(add(sm.c0, sm.c1), add(m0, l3)), v0), v1),
                  add(mul(sm.c2, m0), v1)};
  return {add(f.c0, mul_v(t1)), sub(sub(t2, f.c0), t1)};
}

template <int K>
__device__ __forceinline__ void accum_n_step(Fp12 &f, const uint4 *__restrict__ img, const uint32_t *__restrict__ UV,
                                             int64_t m, int s, int64_t qbase, int64_t pbase, uint32_t live) {
#pragma unroll 1
  for (int k = 0; k < K; k++) {
    if ((live >> k) & 1u) {
      Fp2 a, b;
      load_ab(img, m, s, qbase + (int64_t)k * kWG, a, b);
      const G1A uv = at<G1A>(UV, pbase + (int64_t)k * kWG);  // (u, v) = (x/y, 1/y)
      f = mul_line1(f, mul_fp(a, uv.x), mul_fp(b, uv.y));
    }
  }
}

// as rp_accum_p_kernel, over the normalised image and (u, v) point images
template <int K>
__global__ void __launch_bounds__(kWG) FOLD_OCC rp_accum_n_kernel(const uint4 *__restrict__ img,
                                                                const uint32_t *__restrict__ UV,
                                                                const uint32_t *__restrict__ V_aff, uint32_t *f_blk,
                                                                int64_t m, int64_t period, int G) {
  __shared__ Fp12 sf[kWG / 2];
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x, slot = b >> 3;
  const int v = (int)(slot % G);
  const int64_t qb = (slot / G) * 8 + (b & 7);
  const int64_t qbase = qb * kWG * K + lane, pbase = (int64_t)v * period + qbase;
  uint32_t live = 0;
#pragma unroll 1
  for (int k = 0; k < K; k++) {
    const int64_t q = qbase + (int64_t)k * kWG;
    if (q < m && !at<G1A>(UV, pbase + (int64_t)k * kWG).is_inf() && !at<G2A>(V_aff, q).is_inf()) live |= 1u << k;
  }
  Fp12 f = Fp12::one();
  int s = 0;
  for (int i = ATE_NAF_LEN - 2; i >= 0; i--) {
    if (i != ATE_NAF_LEN - 2) f = sqr(f);
    accum_n_step<K>(f, img, UV, m, s++, qbase, pbase, live);
    if (ATE_NAF[i] != 0) accum_n_step<K>(f, img, UV, m, s++, qbase, pbase, live);
  }
  accum_n_step<K>(f, img, UV, m, s++, qbase, pbase, live);
  accum_n_step<K>(f, img, UV, m, s++, qbase, pbase, live);
  for (int h = kWG / 2; h > 0; h >>= 1) {
    if (lane >= h && lane < 2 * h) sf[lane - h] = f;
    __syncthreads();
    if (lane < h) f = mul(f, sf[lane]);
    __syncthreads();
  }
  if (lane == 0) at<Fp12>(f_blk, (int64_t)v * (period / ((int64_t)kWG * K)) + qb) = f;
}

// G1 side of the fold, one launch per VN: P_it = affine(rho_it (ZB[p*L+j] -
// Y[p*S+i])) for it = (p*S + i)*L + j -- the gather, the point difference, a
// 3-bit-window multiplication by the 64-bit batch weight (window table in
// LDS, as g1_varmul_kernel) and the affine conversion, fused (no [n]
// intermediates in HBM).
constexpr int kPW = 3, kPE = (1 << kPW) - 1;
__global__ void __launch_bounds__(kWG) DX_OCC rp_points_kernel(const uint32_t *__restrict__ ZB,
                                                               const uint32_t *__restrict__ Yj,
                                                               const uint32_t *__restrict__ rho,
                                                               uint32_t *__restrict__ P_aff, int64_t n, int S, int L) {
  __shared__ uint32_t tab[kPE][24][kWG];
  const int lane = threadIdx.x;
  const int64_t it = (int64_t)blockIdx.x * kWG + lane;
  const int64_t ii = it < n ? it : n - 1;  // tail lanes recompute the last item (never stored)
  const int64_t j = ii % L, pi = ii / L, p = pi / S;
  G1J T = at<G1J>(ZB, p * L + j);
  G1J y = at<G1J>(Yj, pi);
  if (!y.is_inf()) {
    y.y = fneg(y.y);
    g1_add_i(T, y);
  }
  G1J acc = T;
  for (int e = 0; e < kPE; e++) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(&acc);
#pragma unroll
    for (int l = 0; l < 24; l++) tab[e][l][lane] = w[l];
    if (e + 1 < kPE && !T.is_inf()) g1_add_i(acc, T);
  }
  const uint32_t *k = rho + 8 * ii;
  auto digit = [&](int wdx) -> uint32_t {
    const int bit = wdx * kPW;
    uint32_t v = k[bit >> 5] >> (bit & 31);
    if ((bit & 31) + kPW > 32 && (bit >> 5) + 1 < 8) v |= k[(bit >> 5) + 1] << (32 - (bit & 31));
    return v & ((1u << kPW) - 1);
  };
  int top = (256 + kPW - 1) / kPW - 1;
  while (top > 0 && digit(top) == 0) top--;
  G1J r = G1J::inf();
  if (!T.is_inf()) {
    for (int wdx = top; wdx >= 0; wdx--) {
#pragma unroll
      for (int d = 0; d < kPW; d++) g1_dbl_i(r);
      const uint32_t dg = digit(wdx);
      if (dg) {
        G1J q;
        uint32_t *w = reinterpret_cast<uint32_t *>(&q);
#pragma unroll
        for (int l = 0; l < 24; l++) w[l] = tab[dg - 1][l][lane];
        g1_add_i(r, q);
      }
    }
  }
  if (it < n) at<G1A>(P_aff, it) = to_affine(r);
}

template <int K>
__device__ __forceinline__ void accum_step(Fp12 &f, const uint4 *__restrict__ lines, int64_t n, int s, int64_t base) {
#pragma unroll 1
  for (int k = 0; k < K; k++) {
    const int64_t it = base + (int64_t)k * kWG;
    if (it < n) {
      Fp2 l0, l1, l3;
      load_line(lines, n, s, it, l0, l1, l3);
      f = mul_line(f, l0, l1, l3);
    }
  }
}

// Lane `lane` of workgroup b owns items b*64*K + k*64 + lane (k < K): each
// uint4 load of a step is one contiguous 1 KiB wave access.
template <int K>
__global__ void __launch_bounds__(kWG) FOLD_OCC rp_accum_kernel(const uint4 *__restrict__ lines, uint32_t *f_blk,
                                                              int64_t n) {
  __shared__ Fp12 sf[kWG / 2];
  const int lane = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * kWG * K + lane;
  Fp12 f = Fp12::one();
  int s = 0;
  for (int i = ATE_NAF_LEN - 2; i >= 0; i--) {
    if (i != ATE_NAF_LEN - 2) f = sqr(f);
    accum_step<K>(f, lines, n, s++, base);
    if (ATE_NAF[i] != 0) accum_step<K>(f, lines, n, s++, base);
  }
  accum_step<K>(f, lines, n, s++, base);
  accum_step<K>(f, lines, n, s++, base);
  for (int h = kWG / 2; h > 0; h >>= 1) {
    if (lane >= h && lane < 2 * h) sf[lane - h] = f;
    __syncthreads();
    if (lane < h) f = mul(f, sf[lane]);
    __syncthreads();
  }
  if (lane == 0) at<Fp12>(f_blk, blockIdx.x) = f;
}

}  // namespace

extern "C" {
int FOLD_NAME(dx_fold_steps_)() { return FOLD_NAME(fold_ns_)::kSteps; }

int FOLD_NAME(dx_rp_lines_)(void *stream, const uint32_t *P_aff, const uint32_t *V_aff, uint32_t *lines, int64_t n,
                            int64_t period, int64_t n_v) {
  using namespace FOLD_NAME(fold_ns_);
  if (n <= 0 || period <= 0 || n_v <= 0 || n_v > period) return n <= 0 ? 0 : -2;
  const int64_t blocks = (n + kWG - 1) / kWG;
  hipLaunchKernelGGL(rp_lines_kernel, dim3((unsigned)blocks), dim3(kWG), 0, (hipStream_t)stream, P_aff, V_aff,
                     reinterpret_cast<uint4 *>(lines), n, period, n_v);
  return check_hip(hipGetLastError(), "rp_lines");
}

int FOLD_NAME(dx_rp_points_)(void *stream, const uint32_t *ZB_jac, const uint32_t *Y_jac, const uint32_t *rho,
                             uint32_t *P_aff, int64_t n, int S, int L) {
  using namespace FOLD_NAME(fold_ns_);
  if (n <= 0) return 0;
  const int64_t blocks = (n + kWG - 1) / kWG;
  hipLaunchKernelGGL(rp_points_kernel, dim3((unsigned)blocks), dim3(kWG), 0, (hipStream_t)stream, ZB_jac, Y_jac, rho,
                     P_aff, n, S, L);
  return check_hip(hipGetLastError(), "rp_points");
}

int FOLD_NAME(dx_rp_coeffs_)(void *stream, const uint32_t *V_aff, uint32_t *coef, int64_t m) {
  using namespace FOLD_NAME(fold_ns_);
  if (m <= 0) return 0;
  const int64_t blocks = (m + kWG - 1) / kWG;
  hipLaunchKernelGGL(rp_coeffs_kernel, dim3((unsigned)blocks), dim3(kWG), 0, (hipStream_t)stream, V_aff,
                     reinterpret_cast<uint4 *>(coef), m);
  return check_hip(hipGetLastError(), "rp_coeffs");
}

// f_blk: G * period / (64 K) Fp12 partial products, verifier-major.
// (Taking a lane's items two at a time -- two sparse lines multiplied
// together first, 23 Fp2 products instead of 26 -- was measured 7% SLOWER:
// more spills; profiles/r2/fold_bench_pair_ab.log.)
int FOLD_NAME(dx_rp_accum_p_)(void *stream, const uint32_t *coef, const uint32_t *P_aff, const uint32_t *V_aff,
                              uint32_t *f_blk, int64_t m, int64_t period, int G, int K) {
  using namespace FOLD_NAME(fold_ns_);
  if (m <= 0 || G <= 0) return 0;
  if (period < m || period % ((int64_t)kWG * K * 8) != 0) return -2;
  const int64_t blocks = (int64_t)G * (period / ((int64_t)kWG * K));
  const uint4 *C = reinterpret_cast<const uint4 *>(coef);
  hipStream_t st = (hipStream_t)stream;
switch (K) {
    case 1: hipLaunchKernelGGL(rp_accum_p_kernel<1>, dim3((unsigned)blocks), dim3(kWG), 0, st, C, P_aff, V_aff, f_blk, m, period, G); break;
    case 2: hipLaunchKernelGGL(rp_accum_p_kernel<2>, dim3((unsigned)blocks), dim3(kWG), 0, st, C, P_aff, V_aff, f_blk, m, period, G); break;
    case 4: hipLaunchKernelGGL(rp_accum_p_kernel<4>, dim3((unsigned)blocks), dim3(kWG), 0, st, C, P_aff, V_aff, f_blk, m, period, G); break;
    case 8: hipLaunchKernelGGL(rp_accum_p_kernel<8>, dim3((unsigned)blocks), dim3(kWG), 0, st, C, P_aff, V_aff, f_blk, m, period, G); break;
    default: return -2;
  }
  return check_hip(hipGetLastError(), "rp_accum_p");
}

// normalised image [steps * 8 * m] uint4 (+ scratch 2 x [steps * 4 * m] uint4)
int FOLD_NAME(dx_rp_ncoeffs_)(void *stream, const uint32_t *V_aff, uint32_t *img, uint32_t *scratch, int64_t m) {
  using namespace FOLD_NAME(fold_ns_);
  if (m <= 0) return 0;
  const int64_t blocks = (m + kWG - 1) / kWG;
  uint4 *sc = reinterpret_cast<uint4 *>(scratch);
  hipLaunchKernelGGL(rp_ncoeffs_kernel, dim3((unsigned)blocks), dim3(kWG), 0, (hipStream_t)stream, V_aff,
                     reinterpret_cast<uint4 *>(img), sc, sc + (int64_t)kSteps * 4 * m, m);
  return check_hip(hipGetLastError(), "rp_ncoeffs");
}

int FOLD_NAME(dx_rp_accum_n_)(void *stream, const uint32_t *img, const uint32_t *UV, const uint32_t *V_aff,
                              uint32_t *f_blk, int64_t m, int64_t period, int G, int K) {
  using namespace FOLD_NAME(fold_ns_);
  if (m <= 0 || G <= 0) return 0;
  if (period < m || period % ((int64_t)kWG * K * 8) != 0) return -2;
  const int64_t blocks = (int64_t)G * (period / ((int64_t)kWG * K));
  const uint4 *C = reinterpret_cast<const uint4 *>(img);
  hipStream_t st = (hipStream_t)stream;
  switch (K) {
    case 1: hipLaunchKernelGGL(rp_accum_n_kernel<1>, dim3((unsigned)blocks), dim3(kWG), 0, st, C, UV, V_aff, f_blk, m, period, G); break;
    case 2: hipLaunchKernelGGL(rp_accum_n_kernel<2>, dim3((unsigned)blocks), dim3(kWG), 0, st, C, UV, V_aff, f_blk, m, period, G); break;
    case 4: hipLaunchKernelGGL(rp_accum_n_kernel<4>, dim3((unsigned)blocks), dim3(kWG), 0, st, C, UV, V_aff, f_blk, m, period, G); break;
    case 8: hipLaunchKernelGGL(rp_accum_n_kernel<8>, dim3((unsigned)blocks), dim3(kWG), 0, st, C, UV, V_aff, f_blk, m, period, G); break;
    default: return -2;
  }
  return check_hip(hipGetLastError(), "rp_accum_n");
}

// f_blk: ceil(n / (64 K)) Fp12 partial products.
int FOLD_NAME(dx_rp_accum_)(void *stream, const uint32_t *lines, uint32_t *f_blk, int64_t n, int K) {
  using namespace FOLD_NAME(fold_ns_);
  if (n <= 0) return 0;
  const int64_t blocks = (n + (int64_t)kWG * K - 1) / ((int64_t)kWG * K);
  const uint4 *L = reinterpret_cast<const uint4 *>(lines);
  hipStream_t st = (hipStream_t)stream;
  switch (K) {
    case 1: hipLaunchKernelGGL(rp_accum_kernel<1>, dim3((unsigned)blocks), dim3(kWG), 0, st, L, f_blk, n); break;
    case 2: hipLaunchKernelGGL(rp_accum_kernel<2>, dim3((unsigned)blocks), dim3(kWG), 0, st, L, f_blk, n); break;
    case 4: hipLaunchKernelGGL(rp_accum_kernel<4>, dim3((unsigned)blocks), dim3(kWG), 0, st, L, f_blk, n); break;
    case 8: hipLaunchKernelGGL(rp_accum_kernel<8>, dim3((unsigned)blocks), dim3(kWG), 0, st, L, f_blk, n); break;
    default: return -2;
  }
  return check_hip(hipGetLastError(), "rp_accum");
}
}  // extern "C"
