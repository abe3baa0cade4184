// GT (Fp12) product chains with THREE lanes per item (device code only).
//
// f = a0 + a1 w over Fp6; Karatsuba needs the three Fp6 products
//   t0 = a0 b0,  t1 = a1 b1,  t2 = (a0 + a1)(b0 + b1)
// and returns c0 = t0 + v t1, c1 = t2 - t0 - t1.  Lane role r of a triple
// holds ONE Fp6 operand -- r0: a0, r1: a1, r2: a0 + a1 -- computes ONE Fp6
// product, and after two 48-dword lane shuffles (ds_bpermute) rebuilds its
// role's operand of the product:
//   r0: c0 = t0 + v t1,   r1: c1 = t2 - t0 - t1,   r2: c0 + c1 = t2 + v t1 - t1.
// One lane holding the whole accumulator, the operand and the Karatsuba
// temporaries needs ~700 registers and spills 1-2 KiB per lane at 2 waves
// per SIMD; a role lane fits in 255 registers with no scratch.  Measured on
// one MI355X (tools/fp12_coop_bench.hip, 993,600 chains of 34 products):
// 22.2 ms against 28.1 ms for the one-lane layout, results bit-identical.
//
// Layout: 21 triples per 64-lane wave (lane 63 idle).  Every lane of a wave
// must reach every shuffle: kernels keep dead triples in the loop (with a
// neutral operand) instead of returning early.
#pragma once
#include "tower.h"

namespace dx {
namespace coop {

constexpr int kTriples = 21;  // items per 64-lane wave

struct Role {
  int r;     // 0, 1, 2
  int base;  // wave lane of the triple's role 0
  int g;     // triple index in the wave (0..20; 21 = the idle lane)
};

__device__ __forceinline__ Role role() {
  const int lane = threadIdx.x & 63;
  const int g = lane / 3;
  return {lane - 3 * g, 3 * g, g};
}

__device__ __forceinline__ Fp6 sel6(bool c, const Fp6 &a, const Fp6 &b) {
  Fp6 out;
  const uint32_t *pa = &a.c0.c0.v[0], *pb = &b.c0.c0.v[0];
  uint32_t *po = &out.c0.c0.v[0];
#pragma unroll
  for (int i = 0; i < 48; i++) po[i] = c ? pa[i] : pb[i];
  return out;
}

// value of `a` in lane `src` of the same wave (src taken modulo 64)
__device__ __forceinline__ Fp6 shfl6(const Fp6 &a, int src) {
  Fp6 out;
  const uint32_t *pa = &a.c0.c0.v[0];
  uint32_t *po = &out.c0.c0.v[0];
#pragma unroll
  for (int i = 0; i < 48; i++) po[i] = (uint32_t)__shfl((int)pa[i], src & 63, 64);
  return out;
}

// role operand of the GT element 1
__device__ __forceinline__ Fp6 one(const Role &R) { return R.r == 1 ? Fp6::zero() : Fp6::one(); }

// role operand of *b (cj: of conj(*b) = b0 - b1 w, the inverse of a unitary b)
__device__ __forceinline__ Fp6 load(const Fp12 *b, bool cj, const Role &R) {
  const Fp6 y0 = R.r != 1 ? b->c0 : Fp6::zero();
  const Fp6 y1 = R.r != 0 ? b->c1 : Fp6::zero();
  return cj ? sub(y0, y1) : add(y0, y1);
}

// tower.h's Karatsuba Fp6 product, force-inlined whatever DX_NI is in the
// including translation unit (an out-of-line call costs spills at the ABI)
__device__ __forceinline__ Fp6 mul6(const Fp6 &a, const Fp6 &b) {
  Fp2 t0 = dx::mul(a.c0, b.c0), t1 = dx::mul(a.c1, b.c1), t2 = dx::mul(a.c2, b.c2);
  Fp2 c0 = add(t0, mul_xi(sub(sub(dx::mul(add(a.c1, a.c2), add(b.c1, b.c2)), t1), t2)));
  Fp2 c1 = add(sub(sub(dx::mul(add(a.c0, a.c1), add(b.c0, b.c1)), t0), t1), mul_xi(t2));
  Fp2 c2 = add(sub(sub(dx::mul(add(a.c0, a.c2), add(b.c0, b.c2)), t0), t2), t1);
  return {c0, c1, c2};
}

// x <- role operand of the product whose role Fp6 products are t
// (t0 = a0 b0 on role 0, t1 = a1 b1 on role 1, t2 = (a0 + a1)(b0 + b1) on role 2)
__device__ __forceinline__ void combine(Fp6 &x, const Fp6 &t, const Role &R) {
  const int lane0 = R.base;
  const Fp6 p = shfl6(t, lane0 + (R.r == 1 ? 0 : 1));  // r0, r2: t1 ; r1: t0
  const Fp6 q = shfl6(t, lane0 + 2);                   // r1: t2
  const Fp6 u = add(t, mul_v(p));                      // r0: c0 ; r2: t2 + v t1
  x = sub(sub(sel6(R.r == 1, q, u), sel6(R.r == 0, Fp6::zero(), p)), sel6(R.r == 1, t, Fp6::zero()));
}

// x <- role operand of (x * y) (x, y: role operands of two GT elements)
__device__ __forceinline__ void mul(Fp6 &x, const Fp6 &y, const Role &R) { combine(x, mul6(x, y), R); }

// Fp6 product with b.c2 = 0 (5 Fp2 products instead of 6)
__device__ __forceinline__ Fp6 mul6_b2z(const Fp6 &a, const Fp6 &b) {
  const Fp2 t0 = dx::mul(a.c0, b.c0), t1 = dx::mul(a.c1, b.c1);
  return {add(t0, mul_xi(dx::mul(a.c2, b.c1))), sub(sub(dx::mul(add(a.c0, a.c1), add(b.c0, b.c1)), t0), t1),
          add(dx::mul(a.c2, b.c0), t1)};
}

// x <- role operand of (x * y) for a y whose role operands all have c2 = 0
// (a sparse Miller line 1 + l1 w + l3 w^3 = 1 + (l1 + l3 v) w: roles (1, 0, 0),
// (l1, l3, 0), (1 + l1, l3, 0))
__device__ __forceinline__ void mul_sparse(Fp6 &x, const Fp6 &y, const Role &R) { combine(x, mul6_b2z(x, y), R); }

// x <- role operand of frob<1>(x): coefficient-wise on the roles 0 and 1
// (conjugation times gamma_1[e], e = the w-exponent), role 2 re-summed
__device__ __forceinline__ void frob1(Fp6 &x, const Role &R) {
  const int o = R.r == 1 ? 1 : 0;  // role 1 holds the odd w-exponents
  auto f = [&](const Fp2 &a, int e) { return dx::mul(conj(a), Fp2::from_limbs(Frob::G1[e])); };
  x = {f(x.c0, o), f(x.c1, 2 + o), f(x.c2, 4 + o)};
  const Fp6 s0 = shfl6(x, R.base), s1 = shfl6(x, R.base + 1);
  if (R.r == 2) x = add(s0, s1);
}

// the full element from the roles 0 / 1 (written by those two lanes)
__device__ __forceinline__ void store(Fp12 *out, const Fp6 &x, const Role &R) {
  if (R.r == 0) out->c0 = x;
  if (R.r == 1) out->c1 = x;
}

}  // namespace coop
}  // namespace dx
