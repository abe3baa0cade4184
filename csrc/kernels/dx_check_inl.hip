// Validity checks of prover-supplied points on the verifier's path (range-proof
// V_ij / combined U_pi in G2, a_ij in the cyclotomic subgroup), compiled with
// every tower and curve function force-inlined into explicit kernels.
//
// Through the generic lambda runner (exec.h) these bodies called the
// out-of-line group law / Fp12 functions of their translation unit, whose call
// frames lived in scratch: 2,396 B per lane for g2_subgroup and 2,528 B for
// gt_cyclotomic (profiles/r5/kernel_resources.txt).  Inlined, the whole check
// stays in registers (tools/kernel_resources.py: 0 B).
#define DX_NI __host__ __device__ __forceinline__
#include "common.h"

using namespace dxk;

namespace {
constexpr int kWG = 64;

// psi on Jacobian coordinates: (X, Y, Z) -> (conj(X) twx, conj(Y) twy, conj(Z)).
DX_HD G2J psi_jac(const G2J &q) {
  return {mul(conj(q.x), Fp2::from_limbs(Frob::TWX1)), mul(conj(q.y), Fp2::from_limbs(Frob::TWY1)), conj(q.z)};
}

// G2 membership of a twist point: on the curve and
//   [u+1] Q + psi([u] Q) + psi^2([u] Q) == psi^3([2u] Q)
// (the BN-curve test of Dai-Lin-Zhao-Zhou 2022: one 63-bit ladder [u] Q instead
// of the 127-bit [6u^2] Q of psi(Q) == [6u^2] Q).  Exact: the cofactor 2p - r is
// squarefree (10069 * 5864401 * 1875725156269 * p54), psi acts on each cyclic
// prime-order part as a scalar, and the test's endomorphism is non-zero on each
// (tests/test_range_hardening.py checks a point of every torsion order).
DX_HD uint8_t g2_subgroup_one(const G2A &q) {
  if (!on_curve(q)) return 0;
  if (q.is_inf()) return 1;
  G2J uq = G2J::from_aff(q);  // top bit of u (bit 62)
  for (int b = 61; b >= 0; --b) {
    uq = jdbl(uq);
    if ((BN_U >> b) & 1ull) uq = jadd_mixed(uq, q);
  }
  const G2J p1 = psi_jac(uq);
  const G2J lhs = jadd(jadd(jadd_mixed(uq, q), p1), psi_jac(p1));
  const G2J rhs = psi_jac(psi_jac(psi_jac(jdbl(uq))));
  return jeq(lhs, rhs) ? 1 : 0;
}

// Membership of the cyclotomic subgroup G_Phi12 (order Phi12(p) = p^4 - p^2 + 1
// = r h): x^(p^4) x == x^(p^2), x != 0 -- two p^2-Frobenius maps (Fp-constant
// coefficient products) and one Fp12 product.  The prime-order part is then
// enforced by the batch equation plus one random combination checked in GT
// (range_proof.py).
DX_HD uint8_t gt_cyclotomic_one(const Fp12 &x) {
  const Fp12 x2 = frob<2>(x);
  return (mul(frob<2>(x2), x) == x2 && !(x.c0 == Fp6::zero() && x.c1 == Fp6::zero())) ? 1 : 0;
}

__global__ void __launch_bounds__(kWG) DX_OCC g2_subgroup_kernel(const uint32_t *aff, uint8_t *out, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (i < n) out[i] = g2_subgroup_one(at<G2A>(aff, i));
}
__global__ void __launch_bounds__(kWG) DX_OCC gt_cyclotomic_kernel(const uint32_t *a, uint8_t *out, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (i < n) out[i] = gt_cyclotomic_one(at<Fp12>(a, i));
}

inline dim3 grid_of(int64_t n) { return dim3((unsigned)((n + kWG - 1) / kWG)); }
}  // namespace

extern "C" {

int dx_g2_subgroup(int on_gpu, void *stream, const uint32_t *aff, uint8_t *out, int64_t n) {
  if (n <= 0) return 0;
  if (!on_gpu) {
    host_for_each(n, [=](int64_t i) { out[i] = g2_subgroup_one(at<G2A>(aff, i)); }, 2);
    return 0;
  }
  hipLaunchKernelGGL(g2_subgroup_kernel, grid_of(n), dim3(kWG), 0, (hipStream_t)stream, aff, out, n);
  return check_hip(hipGetLastError(), "g2_subgroup");
}

int dx_gt_cyclotomic(int on_gpu, void *stream, const uint32_t *a, uint8_t *out, int64_t n) {
  if (n <= 0) return 0;
  if (!on_gpu) {
    host_for_each(n, [=](int64_t i) { out[i] = gt_cyclotomic_one(at<Fp12>(a, i)); }, 2);
    return 0;
  }
  hipLaunchKernelGGL(gt_cyclotomic_kernel, grid_of(n), dim3(kWG), 0, (hipStream_t)stream, a, out, n);
  return check_hip(hipGetLastError(), "gt_cyclotomic");
}

}  // extern "C"
