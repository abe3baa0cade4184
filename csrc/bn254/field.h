// BN254 prime-field arithmetic (Fp and Fr), 8 x 32-bit limbs, Montgomery form.
//
// CDNA4 mapping: every limb product is one `v_mad_u64_u32` (32x32+64 -> 64);
// the no-carry CIOS variant is valid because both moduli have top word
// 0x30644e72 < 2^31-1, so the (m*p + t) accumulator never needs a 9th limb.
// One thread owns one field element (8 VGPRs); kernels are thread-per-item.
//
// The same inline functions are compiled for the host (CPU batch path used by
// the control plane and the CPU test-suite) and for gfx950 device kernels.
// Replaces kyber's bn256 gfP (reference: lib/suite.go:10, external kyber).
#pragma once
#include <cstdint>
#include <hip/hip_runtime.h>
#include "constants.h"

#define DX_HD __host__ __device__ __forceinline__
// DX_NI: out-of-line tower/curve functions (small code, shared by the kernels
// of a translation unit).  A TU may predefine it as force-inline to get one
// register-allocated body per kernel instead (dx_fold_inl.hip).
#ifndef DX_NI
#define DX_NI __host__ __device__ __noinline__ inline
#endif
// The Montgomery multiply is force-inlined into device code (register
// allocation across a whole Fp2/Fp6 product) but kept out-of-line on the host,
// where x86 instruction selection of thousands of unrolled 64-bit MACs would
// otherwise dominate build time.
#ifdef __HIP_DEVICE_COMPILE__
#define DX_MUL DX_HD
#else
#define DX_MUL __host__ __device__ __noinline__ inline
#endif

namespace dx {

// Limb add/subtract with carry.  The clang builtins lower to one
// v_add_co/v_addc_co (v_sub_co/v_subb_co) per limb with the carry kept in
// VCC/an SGPR pair; the equivalent 64-bit C++ arithmetic was lowered to ~5
// VALU instructions per limb on gfx950 (materialised 0/1 carries, 64-bit
// adds, s_nop), which made the modular additions cost as much as the
// Montgomery products around them.
DX_HD uint32_t addc32(uint32_t a, uint32_t b, uint32_t &carry) {
  unsigned co;
  const uint32_t r = __builtin_addc(a, b, carry, &co);
  carry = co;
  return r;
}
DX_HD uint32_t subb32(uint32_t a, uint32_t b, uint32_t &borrow) {
  unsigned bo;
  const uint32_t r = __builtin_subc(a, b, borrow, &bo);
  borrow = bo;
  return r;
}

template <class PR>
struct FieldT {
  uint32_t v[8];

  static DX_HD FieldT zero() {
    FieldT r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = 0;
    return r;
  }
  static DX_HD FieldT one() {
    FieldT r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = PR::ONE[i];
    return r;
  }
  static DX_HD FieldT from_limbs(const uint32_t *p) {
    FieldT r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = p[i];
    return r;
  }
  DX_HD bool is_zero() const {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc |= v[i];
    return acc == 0;
  }
  DX_HD bool operator==(const FieldT &o) const {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc |= v[i] ^ o.v[i];
    return acc == 0;
  }
  DX_HD bool operator!=(const FieldT &o) const { return !(*this == o); }
};

// r = a if borrow==0 after t-MOD else t (i.e. conditional subtract of the modulus)
template <class PR>
DX_HD void cond_sub_mod(uint32_t *t) {
  uint32_t s[8];
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = subb32(t[i], PR::MOD[i], borrow);
  // borrow==1 -> t < MOD -> keep t
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = borrow ? t[i] : s[i];
}

template <class PR>
DX_HD FieldT<PR> fadd(const FieldT<PR> &a, const FieldT<PR> &b) {
  FieldT<PR> r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = addc32(a.v[i], b.v[i], c);
  cond_sub_mod<PR>(r.v);
  return r;
}

template <class PR>
DX_HD FieldT<PR> fsub(const FieldT<PR> &a, const FieldT<PR> &b) {
  FieldT<PR> r;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = subb32(a.v[i], b.v[i], br);
  uint32_t mask = 0u - br;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = addc32(r.v[i], PR::MOD[i] & mask, c);
  return r;
}

template <class PR>
DX_HD FieldT<PR> fneg(const FieldT<PR> &a) {
  return fsub(FieldT<PR>::zero(), a);
}

template <class PR>
DX_HD FieldT<PR> fdbl(const FieldT<PR> &a) {
  return fadd(a, a);
}

#ifdef __HIP_DEVICE_COMPILE__
// acc(64) + hi(32) += x * y: one v_mad_u64_u32 whose carry-out (SGPR pair)
// feeds one v_addc_co_u32 -- two instructions per 32x32 partial product
// (the compiler's lowering of the same C++ needs ~5: a 64-bit add for the
// carry word plus register-pair moves).
__device__ __forceinline__ void dx_mac(uint64_t &acc, uint32_t &hi, uint32_t x, uint32_t y) {
  uint64_t cy, unused;
  asm("v_mad_u64_u32 %0, %2, %4, %5, %0\n\t"
      "v_addc_co_u32_e64 %1, %3, %1, 0, %2"
      : "+v"(acc), "+v"(hi), "=&s"(cy), "=&s"(unused)
      : "v"(x), "v"(y));
}

// Two to four MACs in ONE asm statement.  The hazard recognizer pads the
// boundary between two inline-asm statements with an s_nop (it cannot see
// that the next block only reads VGPRs), which cost one issue slot per MAC
// when every MAC was its own statement; inside a statement the mad -> addc
// carry hand-off needs no wait state (validated bit-exact against the oracle).
#define DX_MAC_STEP(X, Y) "v_mad_u64_u32 %0, %2, %" #X ", %" #Y ", %0\n\tv_addc_co_u32_e64 %1, %3, %1, 0, %2\n\t"
// YC = "v": both factors in VGPRs; YC = "s": the second factor is a uniform
// constant (a modulus limb) read from an SGPR, so it occupies no VGPR.
#define DX_MAC_FNS(SUF, YC)                                                                                      \
  __device__ __forceinline__ void dx_mac1##SUF(uint64_t &acc, uint32_t &hi, uint32_t x0, uint32_t y0) {          \
    uint64_t cy, unused;                                                                                         \
    asm(DX_MAC_STEP(4, 5) : "+v"(acc), "+v"(hi), "=&s"(cy), "=&s"(unused) : "v"(x0), YC(y0));                   \
  }                                                                                                              \
  __device__ __forceinline__ void dx_mac2##SUF(uint64_t &acc, uint32_t &hi, uint32_t x0, uint32_t y0, uint32_t x1, \
                                               uint32_t y1) {                                                    \
    uint64_t cy, unused;                                                                                         \
    asm(DX_MAC_STEP(4, 5) DX_MAC_STEP(6, 7)                                                                      \
        : "+v"(acc), "+v"(hi), "=&s"(cy), "=&s"(unused) : "v"(x0), YC(y0), "v"(x1), YC(y1));                    \
  }                                                                                                              \
  __device__ __forceinline__ void dx_mac3##SUF(uint64_t &acc, uint32_t &hi, uint32_t x0, uint32_t y0, uint32_t x1, \
                                               uint32_t y1, uint32_t x2, uint32_t y2) {                          \
    uint64_t cy, unused;                                                                                         \
    asm(DX_MAC_STEP(4, 5) DX_MAC_STEP(6, 7) DX_MAC_STEP(8, 9)                                                    \
        : "+v"(acc), "+v"(hi), "=&s"(cy), "=&s"(unused)                                                          \
        : "v"(x0), YC(y0), "v"(x1), YC(y1), "v"(x2), YC(y2));                                                    \
  }                                                                                                              \
  __device__ __forceinline__ void dx_mac4##SUF(uint64_t &acc, uint32_t &hi, uint32_t x0, uint32_t y0, uint32_t x1, \
                                               uint32_t y1, uint32_t x2, uint32_t y2, uint32_t x3, uint32_t y3) { \
    uint64_t cy, unused;                                                                                         \
    asm(DX_MAC_STEP(4, 5) DX_MAC_STEP(6, 7) DX_MAC_STEP(8, 9) DX_MAC_STEP(10, 11)                                \
        : "+v"(acc), "+v"(hi), "=&s"(cy), "=&s"(unused)                                                          \
        : "v"(x0), YC(y0), "v"(x1), YC(y1), "v"(x2), YC(y2), "v"(x3), YC(y3));                                   \
  }
#define DX_YV(y) "v"(y)
#define DX_YS(y) "s"(y)
DX_MAC_FNS(_vv, DX_YV)
DX_MAC_FNS(_vs, DX_YS)

// Column accumulator that batches queued MACs into 4-MAC asm statements, one
// queue for products of two variables and one for products by a modulus limb.
// Loops around it are fully unrolled, so the counts are compile-time
// constants at every call and the switches fold away.
struct MacQ {
  uint64_t acc = 0;
  uint32_t hi = 0;
  uint32_t xv[4], yv[4], xs[4], ys[4];
  int nv = 0, ns = 0;
  __device__ __forceinline__ void push(uint32_t a, uint32_t b) {
    xv[nv] = a;
    yv[nv] = b;
    if (++nv == 4) flush_v();
  }
  __device__ __forceinline__ void push_mod(uint32_t a, uint32_t modlimb) {
    xs[ns] = a;
    ys[ns] = modlimb;
    if (++ns == 4) flush_s();
  }
  __device__ __forceinline__ void flush_v() {
    switch (nv) {
      case 1: dx_mac1_vv(acc, hi, xv[0], yv[0]); break;
      case 2: dx_mac2_vv(acc, hi, xv[0], yv[0], xv[1], yv[1]); break;
      case 3: dx_mac3_vv(acc, hi, xv[0], yv[0], xv[1], yv[1], xv[2], yv[2]); break;
      case 4: dx_mac4_vv(acc, hi, xv[0], yv[0], xv[1], yv[1], xv[2], yv[2], xv[3], yv[3]); break;
      default: break;
    }
    nv = 0;
  }
  __device__ __forceinline__ void flush_s() {
    switch (ns) {
      case 1: dx_mac1_vs(acc, hi, xs[0], ys[0]); break;
      case 2: dx_mac2_vs(acc, hi, xs[0], ys[0], xs[1], ys[1]); break;
      case 3: dx_mac3_vs(acc, hi, xs[0], ys[0], xs[1], ys[1], xs[2], ys[2]); break;
      case 4: dx_mac4_vs(acc, hi, xs[0], ys[0], xs[1], ys[1], xs[2], ys[2], xs[3], ys[3]); break;
      default: break;
    }
    ns = 0;
  }
  __device__ __forceinline__ void flush() {
    flush_v();
    flush_s();
  }
  // flush, emit the low word of the column, shift the 96-bit accumulator
  __device__ __forceinline__ uint32_t next_column() {
    flush();
    const uint32_t lo = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
    return lo;
  }
};

// Montgomery multiplication on gfx950: finely integrated product scanning
// (column-wise Comba, Montgomery digits m_i folded into the same columns) with
// one 96-bit column accumulator: ~360 VALU instructions per product instead of
// ~900 for the compiler-lowered CIOS loop (measured: +20% Miller loops/s,
// +30% G1 scalar multiplications/s).  A second, interleaved accumulator per
// column was measured slower: these kernels are issue-bound, not
// latency-bound.  a, b < MOD -> result < MOD.
template <class PR>
__device__ __forceinline__ FieldT<PR> fmul(const FieldT<PR> &a, const FieldT<PR> &b) {
  uint32_t m[8], u[8];
  MacQ q;
#pragma unroll
  for (int i = 0; i < 8; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) {
      q.push(a.v[j], b.v[i - j]);
      q.push_mod(m[j], PR::MOD[i - j]);
    }
    q.push(a.v[i], b.v[0]);
    q.flush();
    m[i] = (uint32_t)q.acc * PR::INV;
    q.push_mod(m[i], PR::MOD[0]);
    (void)q.next_column();
  }
#pragma unroll
  for (int i = 8; i < 16; i++) {
#pragma unroll
    for (int j = i - 7; j < 8; j++) {
      q.push(a.v[j], b.v[i - j]);
      q.push_mod(m[j], PR::MOD[i - j]);
    }
    u[i - 8] = q.next_column();
  }
  // result = u + 2^256 * acc < 2 MOD: one conditional subtraction
  uint32_t s[8], br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = subb32(u[i], PR::MOD[i], br);
  const bool keep = ((uint32_t)q.acc == 0) && br;  // u < MOD and no overflow word
  FieldT<PR> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = keep ? u[i] : s[i];
  return r;
}

// Lazy reduction (device): the 512-bit product and the Montgomery reduction
// as separate steps, so an Fp2 product reduces each output coefficient once
// (2 reductions per 3 products instead of 3) and its additions run on the
// unreduced halves without conditional subtractions.
// acc(64) + hi(32) += x: one v_mad_u64_u32 with the inline constant 1.
__device__ __forceinline__ void dx_add32(uint64_t &acc, uint32_t &hi, uint32_t x) {
  uint64_t cy, unused;
  asm("v_mad_u64_u32 %0, %2, %4, 1, %0\n\t"
      "v_addc_co_u32_e64 %1, %3, %1, 0, %2"
      : "+v"(acc), "+v"(hi), "=&s"(cy), "=&s"(unused)
      : "v"(x));
}

// t[16] = a * b for a, b < 2^255 (product scanning, no reduction).
__device__ __forceinline__ void fmul_wide(const uint32_t *a, const uint32_t *b, uint32_t *t) {
  MacQ q;
#pragma unroll
  for (int i = 0; i < 15; i++) {
#pragma unroll
    for (int j = (i > 7 ? i - 7 : 0); j <= (i < 7 ? i : 7); j++) q.push(a[j], b[i - j]);
    t[i] = q.next_column();
  }
  t[15] = (uint32_t)q.acc;
}

// Montgomery reduction t * 2^-256 mod MOD of a 512-bit t < MOD * 2^256
// (product scanning over the m_i * MOD columns) -> result < MOD.
template <class PR>
__device__ __forceinline__ FieldT<PR> fred_wide(const uint32_t *t) {
  uint32_t m[8], u[8];
  MacQ q;
#pragma unroll
  for (int i = 0; i < 8; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) q.push_mod(m[j], PR::MOD[i - j]);
    q.flush();
    dx_add32(q.acc, q.hi, t[i]);
    m[i] = (uint32_t)q.acc * PR::INV;
    q.push_mod(m[i], PR::MOD[0]);
    (void)q.next_column();
  }
#pragma unroll
  for (int i = 8; i < 16; i++) {
#pragma unroll
    for (int j = i - 7; j < 8; j++) q.push_mod(m[j], PR::MOD[i - j]);
    q.flush();
    dx_add32(q.acc, q.hi, t[i]);
    u[i - 8] = q.next_column();
  }
  // (t + m MOD) / 2^256 < 2 MOD: one conditional subtraction
  uint32_t s[8], br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = subb32(u[i], PR::MOD[i], br);
  const bool keep = ((uint32_t)q.acc == 0) && br;
  FieldT<PR> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = keep ? u[i] : s[i];
  return r;
}
#else
// Montgomery multiplication, no-carry CIOS. a*b*2^-256 mod MOD.
template <class PR>
DX_MUL FieldT<PR> fmul(const FieldT<PR> &a, const FieldT<PR> &b) {
  uint32_t t[8];
#pragma unroll
  for (int j = 0; j < 8; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t bi = b.v[i];
    uint64_t x = (uint64_t)a.v[0] * bi + t[0];
    uint32_t A = (uint32_t)(x >> 32);
    uint32_t t0 = (uint32_t)x;
    uint32_t m = t0 * PR::INV;
    uint64_t y = (uint64_t)m * PR::MOD[0] + t0;
    uint32_t C = (uint32_t)(y >> 32);
#pragma unroll
    for (int j = 1; j < 8; j++) {
      x = (uint64_t)a.v[j] * bi + t[j] + A;
      A = (uint32_t)(x >> 32);
      y = (uint64_t)m * PR::MOD[j] + (uint32_t)x + C;
      C = (uint32_t)(y >> 32);
      t[j - 1] = (uint32_t)y;
    }
    t[7] = C + A;
  }
  cond_sub_mod<PR>(t);
  FieldT<PR> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
  return r;
}
#endif

template <class PR>
DX_HD FieldT<PR> fsqr(const FieldT<PR> &a) {
  return fmul(a, a);
}

// a^e for a little-endian 8-limb exponent (square-and-multiply, MSB first).
template <class PR>
DX_NI FieldT<PR> fpow(const FieldT<PR> &a, const uint32_t *e) {
  FieldT<PR> r = FieldT<PR>::one();
  for (int i = 7; i >= 0; i--) {
    for (int b = 31; b >= 0; b--) {
      r = fsqr(r);
      if ((e[i] >> b) & 1u) r = fmul(r, a);
    }
  }
  return r;
}

// Inverse of a Montgomery-form element (a = xR -> x^-1 R), constant time.
// Binary extended GCD with a fixed iteration count and masked updates
// (invariants A = U z, B = V z mod p; B odd; each step shrinks len(A)+len(B)
// by >= 1, so 510 steps reach A = 0, B = 1 from A < p, B = p < 2^254):
// ~510 x ~60 simple VALU ops instead of Fermat's ~310 dependent Montgomery
// products -- the latency that sets to_affine / decryption-table times for
// short vectors.  V = (xR)^-1 as an integer; V * R^3 (Montgomery) = x^-1 R.
template <class PR>
DX_NI FieldT<PR> finv(const FieldT<PR> &a) {
  uint32_t A[8], B[8], U[8], V[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    A[i] = a.v[i];
    B[i] = PR::MOD[i];
    U[i] = 0;
    V[i] = 0;
  }
  U[0] = 1;
  for (int it = 0; it < 510; it++) {
    const uint32_t odd = 0u - (A[0] & 1u);
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) (void)subb32(A[i], B[i], br);
    const uint32_t sw = odd & (0u - br);  // A odd and A < B: swap
#pragma unroll
    for (int i = 0; i < 8; i++) {
      uint32_t t = (A[i] ^ B[i]) & sw;
      A[i] ^= t;
      B[i] ^= t;
      t = (U[i] ^ V[i]) & sw;
      U[i] ^= t;
      V[i] ^= t;
    }
    // if A odd: A -= B; U = U - V mod p
    br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      uint32_t d = subb32(A[i], B[i], br);
      A[i] = (d & odd) | (A[i] & ~odd);
    }
    br = 0;
    uint32_t D[8];
#pragma unroll
    for (int i = 0; i < 8; i++) D[i] = subb32(U[i], V[i], br);
    const uint32_t neg = 0u - br;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      D[i] = addc32(D[i], PR::MOD[i] & neg, c);
      U[i] = (D[i] & odd) | (U[i] & ~odd);
    }
    // A >>= 1 ; U = U / 2 mod p  (U + p < 2^255: no carry out)
#pragma unroll
    for (int i = 0; i < 7; i++) A[i] = (A[i] >> 1) | (A[i + 1] << 31);
    A[7] >>= 1;
    const uint32_t uo = 0u - (U[0] & 1u);
    c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) U[i] = addc32(U[i], PR::MOD[i] & uo, c);
#pragma unroll
    for (int i = 0; i < 7; i++) U[i] = (U[i] >> 1) | (U[i + 1] << 31);
    U[7] >>= 1;
  }
  const FieldT<PR> r2 = FieldT<PR>::from_limbs(PR::R2);
  return fmul(fmul(FieldT<PR>::from_limbs(V), r2), r2);  // V R^4 R^-2 = x^-1 R
}

// canonical integer (limbs, little endian) <-> Montgomery
template <class PR>
DX_HD FieldT<PR> to_mont(const FieldT<PR> &a) {
  return fmul(a, FieldT<PR>::from_limbs(PR::R2));
}
template <class PR>
DX_HD FieldT<PR> from_mont(const FieldT<PR> &a) {
  FieldT<PR> one = FieldT<PR>::zero();
  one.v[0] = 1;
  return fmul(a, one);
}

// Reduce an arbitrary 256-bit integer (little-endian limbs) below MOD.
// Inputs are < 2^256 < 6*MOD, so at most 5 subtractions are needed.
template <class PR>
DX_HD FieldT<PR> reduce_256(const uint32_t *x) {
  FieldT<PR> r = FieldT<PR>::from_limbs(x);
  for (int k = 0; k < 5; k++) cond_sub_mod<PR>(r.v);
  return r;
}

using Fp = FieldT<FpParams>;
using Fr = FieldT<FrParams>;

}  // namespace dx
