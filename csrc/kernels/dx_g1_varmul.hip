// K4: latency-optimised variable-base G1 scalar multiplication.
//
// The ciphertext vectors of a query are only thousands of elements long
// (e.g. 2070 for SPECTF-shaped LR), so x*K (key switching), s*C (obfuscation),
// c*C / c*y (range-proof verification) and the key-switch proof checks are
// latency-bound: a few dozen workgroups, each thread running a 256-bit
// double-and-add chain.  This kernel keeps that chain in VGPRs: all curve
// formulas force-inlined (no call frames in scratch), the 3-bit window table
// (1P..7P, Jacobian) in LDS as a structure-of-arrays image [entry][limb][lane]
// (conflict-free ds_read_b32, 43 KiB per 64-lane workgroup), one mixed
// uniform window schedule (86 windows x (3 doublings + 1 addition)).
#include "common.h"
#include "../bn254/g1_fast.h"
#include "../bn254/glv_split.h"

namespace {
constexpr int kWG = 64;
constexpr int kWin = 3;
constexpr int kEntries = (1 << kWin) - 1;  // 1P .. 7P

__device__ __forceinline__ void lds_store(uint32_t (*tab)[24][kWG], int e, int lane, const G1J &p) {
  const uint32_t *w = reinterpret_cast<const uint32_t *>(&p);
#pragma unroll
  for (int l = 0; l < 24; l++) tab[e][l][lane] = w[l];
}

__device__ __forceinline__ G1J lds_load(uint32_t (*tab)[24][kWG], int e, int lane) {
  G1J p;
  uint32_t *w = reinterpret_cast<uint32_t *>(&p);
#pragma unroll
  for (int l = 0; l < 24; l++) w[l] = tab[e][l][lane];
  return p;
}

__global__ void __launch_bounds__(kWG) DX_OCC g1_varmul_kernel(const uint32_t *__restrict__ pts, int pt_bcast,
                                                         const uint32_t *__restrict__ sc, int k_bcast,
                                                         uint32_t *__restrict__ out, int64_t n) {
  __shared__ uint32_t tab[kEntries][24][kWG];
  const int lane = threadIdx.x;
  const int64_t i = (int64_t)blockIdx.x * kWG + lane;
  const int64_t ii = i < n ? i : n - 1;  // tail lanes recompute the last item (never stored)
  G1J P = reinterpret_cast<const G1J *>(pts)[pt_bcast ? 0 : ii];
  const uint32_t *k = sc + 8 * (k_bcast ? 0 : ii);
  // table: e -> (e+1) P
  G1J acc = P;
  lds_store(tab, 0, lane, acc);
  for (int e = 1; e < kEntries; e++) {
    g1_add_i(acc, P);
    lds_store(tab, e, lane, acc);
  }
  // top non-zero window
  int top = (256 + kWin - 1) / kWin - 1;
  auto digit = [&](int w) -> uint32_t {
    int bit = w * kWin;
    uint32_t v = k[bit >> 5] >> (bit & 31);
    if ((bit & 31) + kWin > 32 && (bit >> 5) + 1 < 8) v |= k[(bit >> 5) + 1] << (32 - (bit & 31));
    return v & ((1u << kWin) - 1);
  };
  while (top > 0 && digit(top) == 0) top--;
  G1J r = G1J::inf();
  for (int w = top; w >= 0; w--) {
#pragma unroll
    for (int d = 0; d < kWin; d++) g1_dbl_i(r);  // Z = 0 stays 0: no branch needed for infinity
    uint32_t dg = digit(w);
    if (dg) g1_add_i(r, lds_load(tab, (int)dg - 1, lane));
  }
  if (i < n) reinterpret_cast<G1J *>(out)[i] = r;
}

__device__ __forceinline__ G1A affine_with(const G1J &q, const Fp &zi) {
  const Fp zi2 = fsqr(zi);
  return {fmul(q.x, zi2), fmul(fmul(q.y, zi2), zi)};
}

// GLV form of the same product: k P = k1 P + k2 phi(P) with 0 <= k1 < 2^128,
// |k2| < 2^128 (glv_split.h, computed in-kernel from the full scalar) -- a
// 64-window ladder (2 doublings per window, one mixed addition per non-zero
// 2-bit digit of each half) over the affine tables {P, 2P, 3P} and
// {phi(+-P), phi(+-2P), phi(+-3P)} held in VGPRs (one inversion, no LDS):
// 128 doublings + <= 128 mixed additions instead of 256 doublings + 86
// Jacobian additions.  The window schedule is uniform (no leading-zero skip).
__global__ void __launch_bounds__(kWG) DX_OCC g1_glvmul_kernel(const uint32_t *__restrict__ pts, int pt_bcast,
                                                             const uint32_t *__restrict__ sc, int k_bcast,
                                                             const uint32_t *__restrict__ beta_m,
                                                             uint32_t *__restrict__ out, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (i >= n) return;
  const G1J T = reinterpret_cast<const G1J *>(pts)[pt_bcast ? 0 : i];
  const uint32_t *kp = sc + 8 * (k_bcast ? 0 : i);
  uint32_t k[8], k1[4], k2[4];
#pragma unroll
  for (int l = 0; l < 8; l++) k[l] = kp[l];
  bool neg2;
  glv_split(k, k1, k2, neg2);
  if (T.is_inf() || (k1[0] | k1[1] | k1[2] | k1[3] | k2[0] | k2[1] | k2[2] | k2[3]) == 0u) {
    reinterpret_cast<G1J *>(out)[i] = G1J::inf();
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
  const G1A P1 = {fmul(A1.x, beta), neg2 ? fneg(A1.y) : A1.y};
  const G1A P2 = {fmul(A2.x, beta), neg2 ? fneg(A2.y) : A2.y};
  const G1A P3 = {fmul(A3.x, beta), neg2 ? fneg(A3.y) : A3.y};
  G1J r = G1J::inf();
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
  reinterpret_cast<G1J *>(out)[i] = r;
}
}  // namespace

extern "C" int dx_g1_mul_glv256(void *stream, const uint32_t *pts_jac, const uint32_t *scalars,
                                const uint32_t *beta_m, uint32_t *out, int64_t n, int pt_bcast, int k_bcast) {
  if (n <= 0) return 0;
  int64_t blocks = (n + kWG - 1) / kWG;
  hipLaunchKernelGGL(g1_glvmul_kernel, dim3((unsigned)blocks), dim3(kWG), 0, (hipStream_t)stream, pts_jac, pt_bcast,
                     scalars, k_bcast, beta_m, out, n);
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

extern "C" int dx_g1_mul_fast(void *stream, const uint32_t *pts_jac, const uint32_t *scalars, uint32_t *out, int64_t n,
                              int pt_bcast, int k_bcast) {
  if (n <= 0) return 0;
  int64_t blocks = (n + kWG - 1) / kWG;
  hipLaunchKernelGGL(g1_varmul_kernel, dim3((unsigned)blocks), dim3(kWG), 0, (hipStream_t)stream, pts_jac, pt_bcast,
                     scalars, k_bcast, out, n);
  return check_hip(hipGetLastError(), "g1_mul_fast");
}
