// Compact ledger form of range-proof payloads: torus (T2) compression of GT
// elements, and x-coordinate compression of G2 points (below).
//
// A GT element is unitary: f = g + h w (g, h in Fp6, w^2 = v) with
// f conj(f) = g^2 - v h^2 = 1.  For h != 0 it is determined by the single Fp6
// element c = (1 + g) / h, and
//   f = (c + w) / (c - w),   i.e.   g = (c^2 + v) / (c^2 - v),  h = 2c / (c^2 - v)
// (c^2 = v would force g = -1, h = 0).  A range-proof payload is ~68% GT
// elements (the A_j = e(V_j, y)^-s gT^t commitments, 384 bytes each); the
// ledger stores them as c (192 bytes): the same proofs in ~2/3 of the bytes
// the VNs copy off the GPU and fdatasync per query.
//
// The ledger must give back exactly what was signed, so an element is only
// compressed when the round trip is exact: canonical limbs, unitary, h != 0
// (``ok`` = 0 otherwise, and the caller stores that list raw).  Both
// directions take one inversion per chunk of up to kChunk elements
// (Montgomery's simultaneous inversion; t2_chunk), so an element costs a few
// hundred Fp multiplications.  Host and device builds (run()); the tower
// functions are force-inlined into this unit's kernels (no call frames).
#define DX_NI __host__ __device__ __forceinline__
#include "common.h"

namespace {
constexpr int kChunk = 8;

DX_HD bool fp_canonical(const uint32_t *w) {
  uint32_t br = 0;
  for (int k = 0; k < 8; k++) (void)subb32(w[k], FpParams::MOD[k], br);
  return br != 0;
}

// c_i = (1 + g_i) / h_i for a chunk of elements [i0, i1); ok_i as above.
// The prefix products of Montgomery's trick are parked in each element's own
// output slot c_i (an Fp6, the size of the output) and read back by the
// reverse pass: no per-chunk arrays in the thread's frame (the array version
// kept 8 Fp6 prefixes there, 3,552 B of scratch per lane).
DX_HD void compress_chunk(const uint32_t *a, uint32_t *c, uint8_t *ok, int64_t i0, int64_t i1) {
  Fp6 acc = Fp6::one();
  uint32_t good = 0;
  for (int64_t i = i0; i < i1; i++) {
    const uint32_t *w = a + 96 * i;
    bool g = true;
    for (int k = 0; k < 12; k++) g = g && fp_canonical(w + 8 * k);
    const Fp12 f = at<Fp12>(a, i);
    g = g && !(f.c1 == Fp6::zero()) && sub(sqr(f.c0), mul_v(sqr(f.c1))) == Fp6::one();
    at<Fp6>(c, i) = acc;
    if (g) {
      good |= 1u << (i - i0);
      acc = mul(acc, f.c1);
    }
  }
  Fp6 inv_all = inv(acc);
  for (int64_t i = i1 - 1; i >= i0; i--) {
    const bool g = (good >> (i - i0)) & 1u;
    ok[i] = g ? 1 : 0;
    if (!g) {
      at<Fp6>(c, i) = Fp6::zero();
      continue;
    }
    const Fp12 f = at<Fp12>(a, i);
    const Fp6 hi = mul(inv_all, at<Fp6>(c, i));
    inv_all = mul(inv_all, f.c1);
    at<Fp6>(c, i) = mul(add(Fp6::one(), f.c0), hi);
  }
}

// f_i = ((c^2 + v) + 2c w) / (c^2 - v); prefixes parked in the w half of a_i
DX_HD void decompress_chunk(const uint32_t *c, uint32_t *a, int64_t i0, int64_t i1) {
  Fp6 acc = Fp6::one();
  const Fp6 v = {Fp2::zero(), Fp2::one(), Fp2::zero()};
  for (int64_t i = i0; i < i1; i++) {
    const Fp6 x = at<Fp6>(c, i);
    at<Fp12>(a, i).c1 = acc;
    acc = mul(acc, sub(sqr(x), v));
  }
  Fp6 inv_all = inv(acc);
  for (int64_t i = i1 - 1; i >= i0; i--) {
    const Fp6 x = at<Fp6>(c, i);
    const Fp6 x2 = sqr(x);
    const Fp6 di = mul(inv_all, at<Fp12>(a, i).c1);
    inv_all = mul(inv_all, sub(x2, v));
    at<Fp12>(a, i) = Fp12{mul(add(x2, v), di), mul(add(x, x), di)};
  }
}
// ---- G2 points (the V_j of a range proof): x plus one flag word
// (bit 0: parity of y's canonical c0, or of c1 when c0 = 0; bit 1: infinity).
// A point compresses when its limbs are canonical and it is on the twist (or
// is the all-zero infinity); y comes back as the square root of x^3 + b' with
// the stored parity (Adj, Rodriguez-Henriquez: Fp2 square root for p = 3 mod 4).
struct SqrtC {
  static constexpr uint32_t E34[8] = {0xb61f3f51u, 0x4f082305u, 0x5a1c72a3u, 0x65e05aa4u,
                                      0xa0605617u, 0x6e14116du, 0xb84c680au, 0x0c19139cu};  // (p - 3) / 4
  static constexpr uint32_t E12[8] = {0x6c3e7ea3u, 0x9e10460bu, 0xb438e546u, 0xcbc0b548u,
                                      0x40c0ac2eu, 0xdc2822dbu, 0x7098d014u, 0x18322739u};  // (p - 1) / 2
};

DX_HD Fp2 pow2(const Fp2 &a, const uint32_t *e) {
  Fp2 r = Fp2::one();
  for (int bit = 255; bit >= 0; bit--) {
    r = sqr(r);
    if ((e[bit >> 5] >> (bit & 31)) & 1u) r = mul(r, a);
  }
  return r;
}

DX_HD uint32_t y_parity(const Fp2 &y) {
  const Fp c0 = from_mont(y.c0);
  return (c0.is_zero() ? from_mont(y.c1).v[0] : c0.v[0]) & 1u;
}

// one square root of a (a square), else false
DX_HD bool sqrt2(const Fp2 &a, Fp2 &out) {
  const Fp2 a1 = pow2(a, SqrtC::E34);
  const Fp2 alpha = mul(a1, mul(a1, a));
  const Fp2 a0 = mul(conj(alpha), alpha);
  const Fp2 m1 = neg(Fp2::one());
  if (a0 == m1) return false;
  const Fp2 x0 = mul(a1, a);
  if (alpha == m1) {
    out = {fneg(x0.c1), x0.c0};  // i * x0
  } else {
    out = mul(pow2(add(Fp2::one(), alpha), SqrtC::E12), x0);
  }
  return true;
}
}  // namespace

extern "C" {
// V [n, 32] affine G2 -> x [n, 16], flag [n] (parity | 2 * infinity), ok [n]
int dx_g2_x_compress(int on_gpu, void *stream, const uint32_t *V, uint32_t *xo, uint32_t *flag, uint8_t *ok,
                     int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) {
    const uint32_t *w = V + 32 * i;
    bool g = true;
    for (int k = 0; k < 4; k++) g = g && fp_canonical(w + 8 * k);
    const G2A P = at<G2A>(V, i);
    for (int k = 0; k < 16; k++) xo[16 * i + k] = w[k];
    if (P.is_inf()) {
      flag[i] = 2u;
      ok[i] = g ? 1 : 0;
      return;
    }
    flag[i] = y_parity(P.y);
    ok[i] = g && on_curve(P) ? 1 : 0;
  };
  return run(on_gpu, stream, n, op, true, "g2_x_compress");
}

// x [n, 16], flag [n] -> V [n, 32]; bad[i] = 1 where x^3 + b' has no root
int dx_g2_x_decompress(int on_gpu, void *stream, const uint32_t *xi, const uint32_t *flag, uint32_t *V,
                       uint8_t *bad, int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) {
    bad[i] = 0;
    if (flag[i] & 2u) {
      at<G2A>(V, i) = G2A::inf();
      return;
    }
    const Fp2 x = at<Fp2>(xi, i);
    Fp2 y;
    if (!sqrt2(add(mul(sqr(x), x), Fp2::from_limbs(Curve::B2)), y)) {
      bad[i] = 1;
      at<G2A>(V, i) = G2A::inf();
      return;
    }
    if (y_parity(y) != (flag[i] & 1u)) y = neg(y);
    at<G2A>(V, i) = G2A{x, y};
  };
  return run(on_gpu, stream, n, op, true, "g2_x_decompress");
}


// Elements per simultaneous inversion: up to kChunk, but no more than keeps
// >= 2 waves per SIMD busy (1,024 SIMDs x 64 lanes x 2).  A ledger payload is
// one DP's ~10^5 GT elements: 8 per lane left 12k lanes -- a fifth of the
// SIMDs, each lane running 8 elements' products back to back (1.37 ms per
// payload, serialized); one per lane spreads them over the chip and pays one
// Fp6 inversion each.  The host path keeps kChunk (few threads).
inline int64_t t2_chunk(int on_gpu, int64_t n) {
  if (!on_gpu) return kChunk;
  const int64_t c = n / (1024 * 64 * 2);
  return c < 1 ? 1 : (c > kChunk ? kChunk : c);
}

// a [n, 96] GT elements (Montgomery limbs) -> c [n, 48], ok [n] (1: c round-trips to a)
int dx_gt_t2_compress(int on_gpu, void *stream, const uint32_t *a, uint32_t *c, uint8_t *ok, int64_t n) {
  const int64_t k = t2_chunk(on_gpu, n);
  const int64_t chunks = (n + k - 1) / k;
  auto op = [=] __host__ __device__(int64_t t) {
    const int64_t i0 = t * k, i1 = i0 + k < n ? i0 + k : n;
    compress_chunk(a, c, ok, i0, i1);
  };
  return run(on_gpu, stream, chunks, op, true, "gt_t2_compress");
}

// c [n, 48] -> a [n, 96]
int dx_gt_t2_decompress(int on_gpu, void *stream, const uint32_t *c, uint32_t *a, int64_t n) {
  const int64_t k = t2_chunk(on_gpu, n);
  const int64_t chunks = (n + k - 1) / k;
  auto op = [=] __host__ __device__(int64_t t) {
    const int64_t i0 = t * k, i1 = i0 + k < n ? i0 + k : n;
    decompress_chunk(c, a, i0, i1);
  };
  return run(on_gpu, stream, chunks, op, true, "gt_t2_decompress");
}
}  // extern "C"
