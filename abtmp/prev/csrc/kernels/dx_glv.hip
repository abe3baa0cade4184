// GLV-structured batch weights for the range-proof verifier (K16).
//
// A batch verifier may draw each equation's weight from ANY set of 2^64
// distinct residues mod r and keep the 2^-64 soundness of small-exponent
// batching (fixing the other weights, at most one value of a bad equation's
// weight cancels its error in the prime-order group).  The verifier uses
//     rho = a + b * lambda  (a, b uniform 32-bit, lambda the eigenvalue of the
//                            G1 endomorphism phi(x, y) = (beta x, y))
// so that
//   G1: rho T = a T + b phi(T): a joint 2-bit-window (Straus) ladder over 32
//       bits -- 32 doublings instead of 64, a 3-entry affine table in VGPRs
//       (no LDS: the 7-entry LDS window table of the 64-bit kernel held 43 KB
//       per 64-lane workgroup, i.e. < 1 wave per SIMD),
//   GT: x^rho = x^a * frob^8(x)^b (p^8 = lambda mod r), so the bucket
//       multi-exponentiation runs over (a, frob^8 a) with 32-bit exponents.
// Reference: lib/range/range_proof.go:504-565 checks each equation alone.
#include "common.h"
#include "../bn254/g1_fast.h"

using namespace dxk;

namespace {
constexpr int kWG = 64;

__device__ __forceinline__ G1A affine_with(const G1J &q, const Fp &zi) {
  const Fp zi2 = fsqr(zi);
  return {fmul(q.x, zi2), fmul(fmul(q.y, zi2), zi)};
}

// P_it = affine((a_it + b_it lambda)(ZB[p*L+j] - Y[p*S+i])), it = (p*S+i)*L+j.
__global__ void __launch_bounds__(kWG) DX_OCC rp_points_glv_kernel(const uint32_t *__restrict__ ZB,
                                                                 const uint32_t *__restrict__ Yj,
                                                                 const uint32_t *__restrict__ ab,
                                                                 const uint32_t *__restrict__ beta_m,
                                                                 uint32_t *__restrict__ P_aff, int64_t n, int S,
                                                                 int L, int uv) {
  const int64_t it = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (it >= n) return;
  const int64_t j = it % L, pi = it / L, p = pi / S;
  G1J T = at<G1J>(ZB, p * L + j);
  G1J y = at<G1J>(Yj, pi);
  if (!y.is_inf()) {
    y.y = fneg(y.y);
    g1_add_i(T, y);
  }
  if (T.is_inf()) {
    at<G1A>(P_aff, it) = G1A{Fp::zero(), Fp::zero()};
    return;
  }
  // T, 2T, 3T (never infinity: prime order r > 3) to affine with one inversion
  G1J T2 = T;
  g1_dbl_i(T2);
  G1J T3 = T2;
  g1_add_i(T3, T);
  const Fp z12 = fmul(T.z, T2.z);
  Fp inv = finv(fmul(z12, T3.z));
  const Fp i3 = fmul(inv, z12);
  inv = fmul(inv, T3.z);
  const G1A A1 = affine_with(T, fmul(inv, T2.z)), A2 = affine_with(T2, fmul(inv, T.z)), A3 = affine_with(T3, i3);
  const Fp beta = Fp::from_limbs(beta_m);
  const uint32_t a = ab[2 * it], b = ab[2 * it + 1];
  G1J r = G1J::inf();
  for (int w = 15; w >= 0; w--) {
    if (w != 15) {
      g1_dbl_i(r);
      g1_dbl_i(r);
    }
    const uint32_t da = (a >> (2 * w)) & 3u, db = (b >> (2 * w)) & 3u;
    if (da) g1_madd_i(r, da == 1u ? A1 : (da == 2u ? A2 : A3));
    if (db) {
      G1A q = db == 1u ? A1 : (db == 2u ? A2 : A3);
      q.x = fmul(q.x, beta);  // phi(q) = (beta x, y)
      g1_madd_i(r, q);
    }
  }
  if (!uv) {
    at<G1A>(P_aff, it) = to_affine(r);
  } else if (r.is_inf()) {
    at<G1A>(P_aff, it) = G1A{Fp::zero(), Fp::zero()};
  } else {  // (x/y, 1/y) = (X Z / Y, Z^3 / Y): the normalised-line fold's point form
    const Fp iy = finv(r.y);
    at<G1A>(P_aff, it) = G1A{fmul(fmul(r.x, r.z), iy), fmul(fmul(fsqr(r.z), r.z), iy)};
  }
}
// out_i = (a_i + b_i lambda) P_i = a_i P_i + b_i phi(P_i) (Jacobian): the same
// joint 2-bit-window ladder over 32-bit halves, for arbitrary points (the
// key-switch / obfuscation batch checks' weighted rows).  p1: one point for all.
__global__ void __launch_bounds__(kWG) DX_OCC g1_mul_glv_kernel(const uint32_t *__restrict__ P,
                                                              const uint32_t *__restrict__ ab,
                                                              const uint32_t *__restrict__ beta_m,
                                                              uint32_t *__restrict__ out, int64_t n, int p1) {
  const int64_t it = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (it >= n) return;
  const G1J T = at<G1J>(P, p1 ? 0 : it);
  const uint32_t a = ab[2 * it], b = ab[2 * it + 1];
  if (T.is_inf() || (a | b) == 0u) {
    at<G1J>(out, it) = G1J::inf();
    return;
  }
  G1J T2 = T;
  g1_dbl_i(T2);
  G1J T3 = T2;
  g1_add_i(T3, T);
  const Fp z12 = fmul(T.z, T2.z);
  Fp inv = finv(fmul(z12, T3.z));
  const Fp i3 = fmul(inv, z12);
  inv = fmul(inv, T3.z);
  const G1A A1 = affine_with(T, fmul(inv, T2.z)), A2 = affine_with(T2, fmul(inv, T.z)), A3 = affine_with(T3, i3);
  const Fp beta = Fp::from_limbs(beta_m);
  G1J r = G1J::inf();
  for (int w = 15; w >= 0; w--) {
    if (w != 15) {
      g1_dbl_i(r);
      g1_dbl_i(r);
    }
    const uint32_t da = (a >> (2 * w)) & 3u, db = (b >> (2 * w)) & 3u;
    if (da) g1_madd_i(r, da == 1u ? A1 : (da == 2u ? A2 : A3));
    if (db) {
      G1A q = db == 1u ? A1 : (db == 2u ? A2 : A3);
      q.x = fmul(q.x, beta);  // phi(q) = (beta x, y)
      g1_madd_i(r, q);
    }
  }
  at<G1J>(out, it) = r;
}
}  // namespace

extern "C" {
int dx_g1_mul_glv(void *stream, const uint32_t *P_jac, const uint32_t *ab, const uint32_t *beta_m, uint32_t *out,
                  int64_t n, int p1) {
  if (n <= 0) return 0;
  const int64_t blocks = (n + kWG - 1) / kWG;
  hipLaunchKernelGGL(g1_mul_glv_kernel, dim3((unsigned)blocks), dim3(kWG), 0, (hipStream_t)stream, P_jac, ab, beta_m,
                     out, n, p1);
  return check_hip(hipGetLastError(), "g1_mul_glv");
}

// uv = 1: the points as (x/y, 1/y) (fold mode 4) instead of affine (x, y)
int dx_rp_points_glv(void *stream, const uint32_t *ZB_jac, const uint32_t *Y_jac, const uint32_t *ab,
                     const uint32_t *beta_m, uint32_t *P_aff, int64_t n, int S, int L, int uv) {
  if (n <= 0) return 0;
  const int64_t blocks = (n + kWG - 1) / kWG;
  hipLaunchKernelGGL(rp_points_glv_kernel, dim3((unsigned)blocks), dim3(kWG), 0, (hipStream_t)stream, ZB_jac, Y_jac,
                     ab, beta_m, P_aff, n, S, L, uv);
  return check_hip(hipGetLastError(), "rp_points_glv");
}

// affine (x, y) -> (x/y, 1/y) in place (infinity stays zeros)
int dx_g1_aff_to_uv(int on_gpu, void *stream, uint32_t *aff, int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) {
    G1A a = at<G1A>(aff, i);
    if (a.is_inf()) return;
    const Fp iy = finv(a.y);
    at<G1A>(aff, i) = G1A{fmul(a.x, iy), iy};
  };
  return run(on_gpu, stream, n, op, true, "g1_aff_to_uv");
}

// out[i] = a[i]^(p^8) (four Frobenius-squared maps; x^(p^8) = x^lambda on GT)
int dx_gt_frob8(int on_gpu, void *stream, const uint32_t *a, uint32_t *out, int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) {
    Fp12 x = at<Fp12>(a, i);
    x = frob<2>(x);
    x = frob<2>(x);
    x = frob<2>(x);
    at<Fp12>(out, i) = frob<2>(x);
  };
  return run(on_gpu, stream, n, op, true, "gt_frob8");
}
}  // extern "C"
