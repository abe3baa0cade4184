// K4: latency-optimised variable-base G1 scalar multiplication.
//
// The ciphertext vectors of a query are only thousands of elements long
// (e.g. 2070 for SPECTF-shaped LR), so x*K (key switching, decryption), s*C
// (obfuscation), c*C / c*y (range-proof verification) and the key-switch
// proof checks are latency-bound: a few dozen workgroups, each thread running
// one scalar multiplication chain.  The chain stays in VGPRs (all curve
// formulas force-inlined, no call frames in scratch) and is halved by the GLV
// endomorphism.  Round 5 replaced the 256-step window-3 kernel (7-entry
// Jacobian table in LDS, 43 KiB per workgroup): 2.55 -> 2.00 ms at 2-12k rows,
// 15.5 -> 6.0 ms at 262k rows (profiles/r5/glv/micro.txt).
#include "common.h"
#include "../bn254/g1_fast.h"
#include "../bn254/glv_split.h"

namespace {
constexpr int kWG = 64;
__device__ __forceinline__ G1A affine_with(const G1J &q, const Fp &zi) {
  const Fp zi2 = fsqr(zi);
  return {fmul(q.x, zi2), fmul(fmul(q.y, zi2), zi)};
}

// k P = k1 P + k2 phi(P) with 0 <= k1 < 2^128, |k2| < 2^128 (glv_split.h,
// computed in-kernel from the full scalar): a 64-window ladder (2 doublings
// per window, one mixed addition per non-zero 2-bit digit of each half) over
// the affine tables {P, 2P, 3P} and {phi(+-P), phi(+-2P), phi(+-3P)} held in
// VGPRs (one inversion, no LDS): 128 doublings + <= 128 mixed additions
// instead of 256 doublings + 86 Jacobian additions.  kPair: the two halves run
// on the two lanes of a lane pair (each 128 doublings + <= 64 additions, then
// one exchange and one addition) -- the latency form for the short vectors
// that leave most SIMDs idle; the single-lane form does half the total work
// for long ones.  The window schedule is uniform (no leading-zero skip).
template <bool kPair>
__global__ void __launch_bounds__(kWG) DX_OCC g1_glvmul_kernel(const uint32_t *__restrict__ pts, int pt_bcast,
                                                             const uint32_t *__restrict__ sc, int k_bcast,
                                                             const uint32_t *__restrict__ beta_m,
                                                             uint32_t *__restrict__ out, int64_t n) {
  const int64_t t = (int64_t)blockIdx.x * kWG + threadIdx.x;
  const int64_t i = kPair ? t >> 1 : t;
  const int h = kPair ? (int)(t & 1) : 0;
  const bool live = i < n;  // both lanes of a pair agree: no early exit before the exchange
  const int64_t ii = live ? i : n - 1;
  const G1J T = reinterpret_cast<const G1J *>(pts)[pt_bcast ? 0 : ii];
  const uint32_t *kp = sc + 8 * (k_bcast ? 0 : ii);
  uint32_t k[8], k1[4], k2[4];
#pragma unroll
  for (int l = 0; l < 8; l++) k[l] = kp[l];
  bool neg2;
  glv_split(k, k1, k2, neg2);
  const bool zero = T.is_inf() || (k1[0] | k1[1] | k1[2] | k1[3] | k2[0] | k2[1] | k2[2] | k2[3]) == 0u;
  // T, 2T, 3T (never infinity for T != inf: prime order r > 3) to affine with one inversion
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
  if constexpr (kPair) {
    // lane 0: k1 over (P, 2P, 3P); lane 1: |k2| over phi(+-P), ...
    const bool ph = h != 0;
    const Fp b = ph ? beta : Fp::one();
    const bool ng = ph && neg2;
    const G1A E1 = {fmul(A1.x, b), ng ? fneg(A1.y) : A1.y};
    const G1A E2 = {fmul(A2.x, b), ng ? fneg(A2.y) : A2.y};
    const G1A E3 = {fmul(A3.x, b), ng ? fneg(A3.y) : A3.y};
    uint32_t kk[4];
#pragma unroll
    for (int l = 0; l < 4; l++) kk[l] = ph ? k2[l] : k1[l];
#pragma unroll
    for (int q = 3; q >= 0; q--) {
      const uint32_t wa = kk[q];
      for (int d = 15; d >= 0; d--) {
        if (q != 3 || d != 15) {
          g1_dbl_i(r);
          g1_dbl_i(r);
        }
        const uint32_t da = (wa >> (2 * d)) & 3u;
        if (da) g1_madd_i(r, da == 1u ? E1 : (da == 2u ? E2 : E3));
      }
    }
    G1J o;
    const uint32_t *rw = reinterpret_cast<const uint32_t *>(&r);
    uint32_t *ow = reinterpret_cast<uint32_t *>(&o);
#pragma unroll
    for (int l = 0; l < 24; l++) ow[l] = (uint32_t)__shfl_xor((int)rw[l], 1);
    if (h != 0 || !live) return;
    if (!o.is_inf()) g1_add_i(r, o);
  } else {
    const G1A P1 = {fmul(A1.x, beta), neg2 ? fneg(A1.y) : A1.y};
    const G1A P2 = {fmul(A2.x, beta), neg2 ? fneg(A2.y) : A2.y};
    const G1A P3 = {fmul(A3.x, beta), neg2 ? fneg(A3.y) : A3.y};
#pragma unroll
    for (int q = 3; q >= 0; q--) {
      const uint32_t wa = k1[q], wb = k2[q];
      for (int d = 15; d >= 0; d--) {
        if (q != 3 || d != 15) {
          g1_dbl_i(r);
          g1_dbl_i(r);
        }
        const uint32_t da = (wa >> (2 * d)) & 3u, db = (wb >> (2 * d)) & 3u;
        if (da) g1_madd_i(r, da == 1u ? A1 : (da == 2u ? A2 : A3));
        if (db) g1_madd_i(r, db == 1u ? P1 : (db == 2u ? P2 : P3));
      }
    }
    if (!live) return;
  }
  reinterpret_cast<G1J *>(out)[i] = zero ? G1J::inf() : r;
}
}  // namespace

// pair: 1 = two lanes per row (latency form), 0 = one lane per row
extern "C" int dx_g1_mul_glv256(void *stream, const uint32_t *pts_jac, const uint32_t *scalars,
                                const uint32_t *beta_m, uint32_t *out, int64_t n, int pt_bcast, int k_bcast,
                                int pair) {
  if (n <= 0) return 0;
  const int64_t threads = pair ? 2 * n : n;
  const int64_t blocks = (threads + kWG - 1) / kWG;
  if (pair)
    hipLaunchKernelGGL(g1_glvmul_kernel<true>, dim3((unsigned)blocks), dim3(kWG), 0, (hipStream_t)stream, pts_jac,
                       pt_bcast, scalars, k_bcast, beta_m, out, n);
  else
    hipLaunchKernelGGL(g1_glvmul_kernel<false>, dim3((unsigned)blocks), dim3(kWG), 0, (hipStream_t)stream, pts_jac,
                       pt_bcast, scalars, k_bcast, beta_m, out, n);
  return check_hip(hipGetLastError(), "g1_mul_glv256");
}

// [n, 9] words: k1 (4), |k2| (4), k2 < 0 -- the decomposition alone (tests)
extern "C" int dx_glv_split(int on_gpu, void *stream, const uint32_t *k, uint32_t *out, int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) {
    uint32_t k1[4], k2[4];
    bool neg2;
    glv_split(k + 8 * i, k1, k2, neg2);
    for (int l = 0; l < 4; l++) {
      out[9 * i + l] = k1[l];
      out[9 * i + 4 + l] = k2[l];
    }
    out[9 * i + 8] = neg2 ? 1u : 0u;
  };
  return run(on_gpu, stream, n, op, true, "glv_split");
}
