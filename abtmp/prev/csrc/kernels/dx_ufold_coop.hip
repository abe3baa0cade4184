// U side of the regrouped range-proof verifier for SMALL batches: the
// multi-Miller accumulation of fold_body.h's rp_accum_p_kernel with THREE
// lanes per item (csrc/bn254/gt_coop.h).
//
// The verifier's U side pairs every U_q = sum_j rho V_(q, j) with -c y_i
// (lib/range/range_proof.go:540-546, regrouped by bilinearity).  A pool
// rank's 1/W slice has ~20k such items for all VNs: one item per lane fills
// 290 wavefronts, a third of the 1024 SIMDs, each running a serial Fp12 chain
// (one squaring + one sparse line product per Miller step).  Here a lane
// triple shares one item: each lane holds one Fp6 role operand of the
// accumulator and computes one Fp6 product per squaring / line product
// (Karatsuba over w), the triple exchanging its products with two lane
// shuffles -- 3x the wavefronts, about half the per-lane chain.  The lines
// are the RAW coefficients of rp_coeffs_kernel (no normalising inversion
// pass: ~45% cheaper to build for a batch this small).  Large batches (the
// whole inbox on one GPU) keep the one-lane normalised accumulation.
//
// Output: the Miller value of every item t = v * period + q (q >= m or an
// infinity point: one), reduced to 64-item blocks by the caller.
#include "common.h"
#include "../bn254/gt_coop.h"

namespace {

constexpr int count_add_steps() {
  int c = 0;
  for (int i = ATE_NAF_LEN - 2; i >= 0; i--) c += ATE_NAF[i] != 0 ? 1 : 0;
  return c;
}
constexpr int kSteps = (ATE_NAF_LEN - 1) + count_add_steps() + 2;  // doublings + NAF additions + 2 Frobenius lines

// raw (un-normalised) line coefficients: image [step][12][m] uint4 of
// (c0, c1, c3) per step; the line at P = (x, y) is c0 y + (c1 x) w + c3 w^3
__device__ __forceinline__ void load_c3(const uint4 *__restrict__ img, int64_t m, int s, int64_t q, Fp2 &c0, Fp2 &c1,
                                        Fp2 &c3) {
  Fp2 *dst[3] = {&c0, &c1, &c3};
#pragma unroll
  for (int c = 0; c < 3; c++) {
    uint32_t *w = reinterpret_cast<uint32_t *>(dst[c]);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint4 v = img[((int64_t)s * 12 + c * 4 + k) * m + q];
      w[4 * k] = v.x;
      w[4 * k + 1] = v.y;
      w[4 * k + 2] = v.z;
      w[4 * k + 3] = v.w;
    }
  }
}

// x <- x * (l0 + l1 w + l3 w^3) on the triple: roles (l0, 0, 0), (l1, l3, 0),
// (l0 + l1, l3, 0); dead items multiply by one
__device__ __forceinline__ void raw_line_step(Fp6 &x, const uint4 *__restrict__ img, int64_t m, int s, int64_t q,
                                              const G1A &P, bool live, const coop::Role &R) {
  Fp2 c0, c1, c3;
  load_c3(img, m, s, q, c0, c1, c3);
  const Fp2 l0 = mul_fp(c0, P.y), l1 = mul_fp(c1, P.x);
  Fp6 y = Fp6::one();
  if (live) y = {R.r == 0 ? l0 : (R.r == 1 ? l1 : add(l0, l1)), R.r == 0 ? Fp2::zero() : c3, Fp2::zero()};
  coop::mul_sparse(x, y, R);
}

// as ufold_coop_kernel over the raw coefficient image and affine points P
// (one item t = v * period + q per triple): a small batch's coefficients
// without the normalising inversion pass (~45% cheaper to build)
__global__ void __launch_bounds__(64) DX_OCC ufold_coop_raw_kernel(const uint4 *__restrict__ img,
                                                                   const uint32_t *__restrict__ P_aff,
                                                                   const uint32_t *__restrict__ V_aff,
                                                                   uint32_t *__restrict__ f_out, int64_t m,
                                                                   int64_t period, int64_t n_items) {
  // item t's product goes to row (t % 64) * (n_items / 64) + t / 64: the
  // [64, n_items / 64] lane-major image the 8-way product levels read
  // contiguously (no transposing copy between the fold and the reduction)
  const coop::Role R = coop::role();
  const int64_t t = (int64_t)blockIdx.x * coop::kTriples + R.g;
  const bool real = R.g < coop::kTriples && t < n_items;
  const int64_t q = real ? t % period : 0;
  const bool in = real && q < m;
  const G1A P = in ? at<G1A>(P_aff, t) : G1A{Fp::zero(), Fp::zero()};
  const bool live = in && !P.is_inf() && !at<G2A>(V_aff, q).is_inf();
  const int64_t qq = live ? q : 0;
  Fp6 x = coop::one(R);
  int s = 0;
  for (int i = ATE_NAF_LEN - 2; i >= 0; i--) {
    if (i != ATE_NAF_LEN - 2) coop::mul(x, x, R);
    raw_line_step(x, img, m, s++, qq, P, live, R);
    if (ATE_NAF[i] != 0) raw_line_step(x, img, m, s++, qq, P, live, R);
  }
  raw_line_step(x, img, m, s++, qq, P, live, R);
  raw_line_step(x, img, m, s++, qq, P, live, R);
  if (real) coop::store(&at<Fp12>(f_out, (t & 63) * (n_items >> 6) + (t >> 6)), x, R);
}

}  // namespace

extern "C" {

// raw coefficient image (kSteps * 12 * m uint4) and affine points P [n_items]
int dx_ufold_coop_raw(void *stream, const uint32_t *img, const uint32_t *P_aff, const uint32_t *V_aff,
                      uint32_t *f_out, int64_t m, int64_t period, int64_t n_items) {
  if (n_items <= 0 || m <= 0 || period < m || n_items % 64) return n_items <= 0 ? 0 : -2;
  const unsigned blocks = (unsigned)((n_items + coop::kTriples - 1) / coop::kTriples);
  hipLaunchKernelGGL(ufold_coop_raw_kernel, dim3(blocks), dim3(64), 0, (hipStream_t)stream,
                     reinterpret_cast<const uint4 *>(img), P_aff, V_aff, f_out, m, period, n_items);
  return check_hip(hipGetLastError(), "ufold_coop_raw");
}

int dx_ufold_coop_steps() { return kSteps; }

}  // extern "C"
