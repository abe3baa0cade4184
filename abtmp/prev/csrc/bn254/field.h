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

// Inverse of a Montgomery-form element (a = xR -> x^-1 R), constant time:
// Bernstein-Yang "safegcd" with half-delta divsteps (the variant and the
// 10 x 59 = 590-step bound for 256-bit moduli of libsecp256k1's modinv64;
// written here from the published algorithm).  The divsteps run on the low
// 64 bits of (f, g) alone, 59 at a time, accumulating a 2x2 transition
// matrix scaled by 2^62; each batch then applies the matrix to the full
// 5 x 62-bit signed limbs of f, g and of the Bezout tracker (d, e) (mod p,
// with a p multiple that clears the low 62 bits before the shift).  Starting
// e at R^2 mod p makes d = R^2 (xR)^-1 = x^-1 R directly.  ~590 x 16 simple
// 64-bit ops plus 10 x 44 64x64 products: ~4x fewer VALU instructions than
// the bitwise binary GCD it replaces (510 steps over 8-limb values).
namespace inv62 {
using i64 = int64_t;
using u64 = uint64_t;
using i128 = __int128;
constexpr u64 M62 = ~0ull >> 2;

// bits [62 k, 62 k + 62) of a little-endian 8 x 32-bit integer
constexpr i64 limb(const uint32_t (&w)[8], int k) {
  u64 r = 0;
  for (int b = 0; b < 62; b++) {
    const int bit = 62 * k + b;
    if (bit < 256 && ((w[bit / 32] >> (bit % 32)) & 1u)) r |= 1ull << b;
  }
  return (i64)r;
}
// p^-1 mod 2^62 (Newton: each step doubles the correct low bits; p odd)
constexpr u64 inv_mod62(const uint32_t (&w)[8]) {
  const u64 p0 = (u64)w[0] | ((u64)w[1] << 32);
  u64 x = p0;  // correct mod 2^3 for odd p
  for (int i = 0; i < 6; i++) x *= 2 - p0 * x;
  return x & M62;
}

DX_HD i64 divsteps59(i64 zeta, u64 f, u64 g, i64 &tu, i64 &tv, i64 &tq, i64 &tr) {
  u64 u = 8, v = 0, q = 0, r = 8;  // identity x 2^3: 59 steps later the matrix carries 2^62
  for (int i = 3; i < 62; i++) {
    u64 m1 = (u64)(zeta >> 63);    // zeta < 0
    const u64 m2 = 0 - (g & 1);    // g odd
    const u64 x = (f ^ m1) - m1, y = (u ^ m1) - m1, z = (v ^ m1) - m1;
    g += x & m2;
    q += y & m2;
    r += z & m2;
    m1 &= m2;                      // zeta < 0 and g odd: swap (f <- g, zeta <- -zeta - 2)
    zeta = (zeta ^ (i64)m1) - 1;
    f += g & m1;
    u += q & m1;
    v += r & m1;
    g >>= 1;
    u <<= 1;
    v <<= 1;
  }
  tu = (i64)u;
  tv = (i64)v;
  tq = (i64)q;
  tr = (i64)r;
  return zeta;
}

// [f, g] <- t [f, g] / 2^62 (exact)
DX_HD void update_fg(i64 *f, i64 *g, i64 u, i64 v, i64 q, i64 r) {
  i128 cf = (i128)u * f[0] + (i128)v * g[0];
  i128 cg = (i128)q * f[0] + (i128)r * g[0];
  cf >>= 62;
  cg >>= 62;
#pragma unroll
  for (int k = 1; k < 5; k++) {
    cf += (i128)u * f[k] + (i128)v * g[k];
    cg += (i128)q * f[k] + (i128)r * g[k];
    f[k - 1] = (i64)((u64)cf & M62);
    g[k - 1] = (i64)((u64)cg & M62);
    cf >>= 62;
    cg >>= 62;
  }
  f[4] = (i64)cf;
  g[4] = (i64)cg;
}

// [d, e] <- (t [d, e] + p [md, me]) / 2^62, md / me chosen so the division is exact
// and d, e stay in (-2p, p)
DX_HD void update_de(i64 *d, i64 *e, i64 u, i64 v, i64 q, i64 r, const i64 *P, u64 pinv) {
  const i64 sd = d[4] >> 63, se = e[4] >> 63;
  i64 md = (u & sd) + (v & se);
  i64 me = (q & sd) + (r & se);
  i128 cd = (i128)u * d[0] + (i128)v * e[0];
  i128 ce = (i128)q * d[0] + (i128)r * e[0];
  md -= (i64)((pinv * (u64)cd + (u64)md) & M62);
  me -= (i64)((pinv * (u64)ce + (u64)me) & M62);
  cd += (i128)P[0] * md;
  ce += (i128)P[0] * me;
  cd >>= 62;
  ce >>= 62;
#pragma unroll
  for (int k = 1; k < 5; k++) {
    cd += (i128)u * d[k] + (i128)v * e[k] + (i128)P[k] * md;
    ce += (i128)q * d[k] + (i128)r * e[k] + (i128)P[k] * me;
    d[k - 1] = (i64)((u64)cd & M62);
    e[k - 1] = (i64)((u64)ce & M62);
    cd >>= 62;
    ce >>= 62;
  }
  d[4] = (i64)cd;
  e[4] = (i64)ce;
}

// d in (-2p, p), negated if sign < 0 -> [0, p)
DX_HD void normalize(i64 *d, i64 sign, const i64 *P) {
  i64 c = d[4] >> 63;
#pragma unroll
  for (int k = 0; k < 5; k++) d[k] += P[k] & c;
  const i64 n = sign >> 63;
#pragma unroll
  for (int k = 0; k < 5; k++) d[k] = (d[k] ^ n) - n;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    d[k + 1] += d[k] >> 62;
    d[k] &= (i64)M62;
  }
  c = d[4] >> 63;
#pragma unroll
  for (int k = 0; k < 5; k++) d[k] += P[k] & c;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    d[k + 1] += d[k] >> 62;
    d[k] &= (i64)M62;
  }
}
}  // namespace inv62

template <class PR>
DX_NI FieldT<PR> finv(const FieldT<PR> &a) {
  using namespace inv62;
  constexpr i64 P0 = limb(PR::MOD, 0), P1 = limb(PR::MOD, 1), P2 = limb(PR::MOD, 2), P3 = limb(PR::MOD, 3),
                P4 = limb(PR::MOD, 4);
  constexpr i64 E0 = limb(PR::R2, 0), E1 = limb(PR::R2, 1), E2 = limb(PR::R2, 2), E3 = limb(PR::R2, 3),
                E4 = limb(PR::R2, 4);
  constexpr u64 PINV = inv_mod62(PR::MOD);
  const i64 P[5] = {P0, P1, P2, P3, P4};
  i64 f[5] = {P0, P1, P2, P3, P4};
  i64 e[5] = {E0, E1, E2, E3, E4};
  i64 d[5] = {0, 0, 0, 0, 0};
  i64 g[5];
  const uint32_t *w = a.v;
  g[0] = (i64)(((u64)w[0] | ((u64)w[1] << 32)) & M62);
  g[1] = (i64)((((u64)w[1] >> 30) | ((u64)w[2] << 2) | ((u64)w[3] << 34)) & M62);
  g[2] = (i64)((((u64)w[3] >> 28) | ((u64)w[4] << 4) | ((u64)w[5] << 36)) & M62);
  g[3] = (i64)((((u64)w[5] >> 26) | ((u64)w[6] << 6) | ((u64)w[7] << 38)) & M62);
  g[4] = (i64)((u64)w[7] >> 24);
  i64 zeta = -1;  // -(delta + 1/2), delta = 1/2
  for (int it = 0; it < 10; it++) {
    i64 u, v, q, r;
    zeta = divsteps59(zeta, (u64)f[0], (u64)g[0], u, v, q, r);
    update_de(d, e, u, v, q, r, P, PINV);
    update_fg(f, g, u, v, q, r);
  }
  normalize(d, f[4], P);  // g = 0, f = +-1: d = +- R^2 a^-1
  FieldT<PR> out;
  out.v[0] = (uint32_t)d[0];
  out.v[1] = (uint32_t)(((u64)d[0] >> 32) | ((u64)d[1] << 30));
  out.v[2] = (uint32_t)((u64)d[1] >> 2);
  out.v[3] = (uint32_t)(((u64)d[1] >> 34) | ((u64)d[2] << 28));
  out.v[4] = (uint32_t)((u64)d[2] >> 4);
  out.v[5] = (uint32_t)(((u64)d[2] >> 36) | ((u64)d[3] << 26));
  out.v[6] = (uint32_t)((u64)d[3] >> 6);
  out.v[7] = (uint32_t)(((u64)d[3] >> 38) | ((u64)d[4] << 24));
  return out;
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
