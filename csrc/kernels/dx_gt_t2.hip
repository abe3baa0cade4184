// Torus (T2) compression of GT elements for the proof ledger.
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
// directions take one inversion per chunk of kChunk elements (Montgomery's
// simultaneous inversion), so a query's ~10^6 elements cost a few hundred
// Fp multiplications each.  Host and device builds (run()).
#include "common.h"

namespace {
constexpr int kChunk = 8;

DX_HD bool fp_canonical(const uint32_t *w) {
  uint32_t br = 0;
  for (int k = 0; k < 8; k++) (void)subb32(w[k], FpParams::MOD[k], br);
  return br != 0;
}

// c_i = (1 + g_i) / h_i for a chunk of elements [i0, i1); ok_i as above
DX_HD void compress_chunk(const uint32_t *a, uint32_t *c, uint8_t *ok, int64_t i0, int64_t i1) {
  Fp6 pre[kChunk];
  Fp6 acc = Fp6::one();
  bool good[kChunk];
  for (int64_t i = i0; i < i1; i++) {
    const int j = (int)(i - i0);
    const uint32_t *w = a + 96 * i;
    bool g = true;
    for (int k = 0; k < 12; k++) g = g && fp_canonical(w + 8 * k);
    const Fp12 f = at<Fp12>(a, i);
    g = g && !(f.c1 == Fp6::zero()) && sub(sqr(f.c0), mul_v(sqr(f.c1))) == Fp6::one();
    good[j] = g;
    pre[j] = acc;
    if (g) acc = mul(acc, f.c1);
  }
  Fp6 inv_all = inv(acc);
  for (int64_t i = i1 - 1; i >= i0; i--) {
    const int j = (int)(i - i0);
    ok[i] = good[j] ? 1 : 0;
    if (!good[j]) {
      at<Fp6>(c, i) = Fp6::zero();
      continue;
    }
    const Fp12 f = at<Fp12>(a, i);
    const Fp6 hi = mul(inv_all, pre[j]);
    inv_all = mul(inv_all, f.c1);
    at<Fp6>(c, i) = mul(add(Fp6::one(), f.c0), hi);
  }
}

// f_i = ((c^2 + v) + 2c w) / (c^2 - v)
DX_HD void decompress_chunk(const uint32_t *c, uint32_t *a, int64_t i0, int64_t i1) {
  Fp6 pre[kChunk];
  Fp6 acc = Fp6::one();
  const Fp6 v = {Fp2::zero(), Fp2::one(), Fp2::zero()};
  for (int64_t i = i0; i < i1; i++) {
    const Fp6 x = at<Fp6>(c, i);
    pre[i - i0] = acc;
    acc = mul(acc, sub(sqr(x), v));
  }
  Fp6 inv_all = inv(acc);
  for (int64_t i = i1 - 1; i >= i0; i--) {
    const Fp6 x = at<Fp6>(c, i);
    const Fp6 x2 = sqr(x);
    const Fp6 di = mul(inv_all, pre[i - i0]);
    inv_all = mul(inv_all, sub(x2, v));
    at<Fp12>(a, i) = Fp12{mul(add(x2, v), di), mul(add(x, x), di)};
  }
}
}  // namespace

extern "C" {
// a [n, 96] GT elements (Montgomery limbs) -> c [n, 48], ok [n] (1: c round-trips to a)
int dx_gt_t2_compress(int on_gpu, void *stream, const uint32_t *a, uint32_t *c, uint8_t *ok, int64_t n) {
  const int64_t chunks = (n + kChunk - 1) / kChunk;
  auto op = [=] __host__ __device__(int64_t t) {
    const int64_t i0 = t * kChunk, i1 = i0 + kChunk < n ? i0 + kChunk : n;
    compress_chunk(a, c, ok, i0, i1);
  };
  return run(on_gpu, stream, chunks, op, true, "gt_t2_compress");
}

// c [n, 48] -> a [n, 96]
int dx_gt_t2_decompress(int on_gpu, void *stream, const uint32_t *c, uint32_t *a, int64_t n) {
  const int64_t chunks = (n + kChunk - 1) / kChunk;
  auto op = [=] __host__ __device__(int64_t t) {
    const int64_t i0 = t * kChunk, i1 = i0 + kChunk < n ? i0 + kChunk : n;
    decompress_chunk(c, a, i0, i1);
  };
  return run(on_gpu, stream, chunks, op, true, "gt_t2_decompress");
}
}  // extern "C"
