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
}  // namespace

extern "C" int dx_g1_mul_fast(void *stream, const uint32_t *pts_jac, const uint32_t *scalars, uint32_t *out, int64_t n,
                              int pt_bcast, int k_bcast) {
  if (n <= 0) return 0;
  int64_t blocks = (n + kWG - 1) / kWG;
  hipLaunchKernelGGL(g1_varmul_kernel, dim3((unsigned)blocks), dim3(kWG), 0, (hipStream_t)stream, pts_jac, pt_bcast,
                     scalars, k_bcast, out, n);
  return check_hip(hipGetLastError(), "g1_mul_fast");
}
