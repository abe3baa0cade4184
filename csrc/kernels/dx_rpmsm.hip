// Range-proof batch verification by bilinearity (K16, verifier mode "msm").
//
// The batched range-proof equation of one verifier (weights rho_it, items
// it = (p*S + i)*L + j: proof p, server i, digit j; reference per-equation
// check lib/range/range_proof.go:504-565) needs
//     prod_it e(rho_it (Zphi_pj B - c_p y_pi), V_it)
// which the Miller fold evaluates as one Miller loop per item.  Bilinearity
// regroups it into
//     e(B, R) * prod_(p,i) e(-Y_pi, U_pi),   Y_pi = c_p y_pi,
//     R    = sum_it (rho_it Zphi_pj) V_it              (one G2 MSM),
//     U_pi = sum_j rho_(p,i,j) V_(p,i,j)                (L-point combinations),
// i.e. n*S + 1 Miller loops instead of n*S*L, for the price of G2 additions:
//   * the verifier's weights are rho = a + b lambda with 32-bit halves (see
//     dx_glv.hip); on G2 [lambda] Q = -psi^2(Q) = (x * TWX2, y) (one Fp2 x Fp
//     product), so U_pi is a joint 2-bit-window ladder over 32 bits in which
//     each (window, digit) adds ONE point da V + db [lambda] V from a
//     15-entry affine table per V (built once, shared by every verifier of
//     the rank): 32 doublings + 16 L mixed additions, the same for every
//     lane of a wave (no NAF divergence);
//   * R is a Pippenger MSM (c-bit windows, bucket plan sorted on the device,
//     segmented bucket sums, bucket weights d B_d, per-window sums and a
//     Horner step per verifier that writes R straight into the Miller-loop
//     input list: no host round trip between the MSM and the pairing fold).
// Soundness: the check is the same equation (bilinearity on G2 x G1); every
// V_it is on the twist (decode check), the combined points are in G2 by
// construction when the V_it are, and a failed batch falls back to the
// per-request re-check (requests.py) that blames the bad request.
#define DX_NI __host__ __device__ __forceinline__
#include "common.h"

using namespace dxk;

namespace {
constexpr int kT = 15;  // table entries per V: da V + db [lambda] V, (da, db) in [0, 3]^2 \ {(0, 0)}

DX_HD G2J lam_jac(const G2J &q) {  // [lambda] Q = -psi^2(Q) = (TWX2 x, y) (TWX2 in Fp)
  return {mul_fp(q.x, Fp::from_limbs(Frob::TWX2[0])), q.y, q.z};
}
// Every device body below is force-inlined into an explicit __global__
// kernel.  Large bodies reached through the generic lambda runner stayed
// out-of-line callees, and branch relaxation in such a callee reused the
// return-address SGPR pair s[30:31] for its long jumps (gfx950 ISA of the first
// version of this file): the kernels here make no calls at all.
constexpr int kWG = 64;

// T[it*15 + da + 4 db - 1] = affine(da V_it + db [lambda] V_it).  2V and 3V
// come from ONE inversion (Jacobian, Montgomery's trick over their two Z);
// the six single-axis entries (da V, db [lambda] V: [lambda] = x * TWX2) are
// then written at once, and the nine mixed entries da V + db [lambda] V are
// AFFINE additions sharing a second inversion: d = x_b - x_a per entry, the
// prefix products parked in the x of each entry's own output slot (read back
// in the reverse pass), the operand points re-read from their slots -- no
// per-entry arrays in the thread's frame (the previous Jacobian version kept
// 15 Z values and prefix products there: 3,360 B of scratch per lane,
// profiles/r5/kernel_resources.txt) and ~1/3 of its field products.
DX_HD void joint_table_one(const uint32_t *V_aff, uint32_t *T_aff, int64_t it) {
  G2A *T = reinterpret_cast<G2A *>(T_aff) + it * kT;
  const G2A v = at<G2A>(V_aff, it);
  if (v.is_inf()) {
    for (int e = 0; e < kT; e++) T[e] = G2A::inf();
    return;
  }
  const Fp tw = Fp::from_limbs(Frob::TWX2[0]);
  {
    const G2J P2 = jdbl(G2J::from_aff(v));
    const G2J P3 = jadd_mixed(P2, v);
    const Fp2 ii = inv(mul(P2.z, P3.z));  // 2V, 3V != infinity (r is prime, > 3)
    const Fp2 z2i = mul(ii, P3.z), z3i = mul(ii, P2.z);
    const Fp2 z2i2 = sqr(z2i), z3i2 = sqr(z3i);
    const G2A A2{mul(P2.x, z2i2), mul(mul(P2.y, z2i2), z2i)};
    const G2A A3{mul(P3.x, z3i2), mul(mul(P3.y, z3i2), z3i)};
    T[0] = v;                                 // (1, 0)
    T[1] = A2;                                // (2, 0)
    T[2] = A3;                                // (3, 0)
    T[3] = G2A{mul_fp(v.x, tw), v.y};         // (0, 1)
    T[7] = G2A{mul_fp(A2.x, tw), A2.y};       // (0, 2)
    T[11] = G2A{mul_fp(A3.x, tw), A3.y};      // (0, 3)
  }
  // mixed entries e = da + 4 db - 1, da, db in 1..3: forward prefix products
  // of d_e = x(db [lambda] V) - x(da V) (nonzero: da V != +-db [lambda] V)
  Fp2 acc = Fp2::one();
  for (int db = 1; db < 4; db++) {
    for (int da = 1; da < 4; da++) {
      const int e = da + 4 * db - 1;
      const Fp2 d = sub(T[4 * db - 1].x, T[da - 1].x);
      T[e].x = acc;  // parked: the prefix product before this entry
      acc = mul(acc, d);
    }
  }
  Fp2 iv = inv(acc);
  for (int db = 3; db >= 1; db--) {
    for (int da = 3; da >= 1; da--) {
      const int e = da + 4 * db - 1;
      const G2A a = T[da - 1], b = T[4 * db - 1];
      const Fp2 d = sub(b.x, a.x);
      const Fp2 di = mul(iv, T[e].x);  // 1 / d_e
      iv = mul(iv, d);
      const Fp2 lm = mul(sub(b.y, a.y), di);
      const Fp2 x3 = sub(sub(sqr(lm), a.x), b.x);
      T[e] = G2A{x3, sub(mul(lm, sub(a.x, x3)), a.y)};
    }
  }
}

// (pos: when given, U of (v, q) goes to row pos[v * n_groups + q] instead of v * pad + q)
DX_HD void u_joint_one(const uint32_t *T_aff, const uint32_t *ab, uint32_t *U_aff, int64_t n_groups, int L,
                       int64_t pad, const int64_t *pos, int64_t t) {
  const int64_t m = n_groups * L;
  const int64_t v = t / n_groups, q = t % n_groups;
  const G2A *T = reinterpret_cast<const G2A *>(T_aff) + q * L * kT;
  const uint32_t *w = ab + 2 * (v * m + q * L);
  G2J acc = G2J::inf();
  for (int win = 15; win >= 0; win--) {
    if (win != 15) {
      acc = jdbl(acc);
      acc = jdbl(acc);
    }
    for (int j = 0; j < L; j++) {
      const uint32_t e = ((w[2 * j] >> (2 * win)) & 3u) + 4u * ((w[2 * j + 1] >> (2 * win)) & 3u);
      if (e) acc = jadd_mixed(acc, T[j * kT + e - 1]);
    }
  }
  at<G2A>(U_aff, pos ? pos[t] : v * pad + q) = to_affine(acc);
}

// The same combination split over sp threads per (v, q) (small batches: a
// pool helper's 1/W slice gives too few (v, q) to fill 256 CUs): part p sums
// digits [p L/sp, (p+1) L/sp) into a Jacobian partial; u_joint_reduce_one adds
// the sp partials and normalises.
DX_HD void u_joint_part_one(const uint32_t *T_aff, const uint32_t *ab, uint32_t *P_jac, int64_t n_groups, int L,
                            int sp, int64_t t) {
  const int64_t m = n_groups * L;
  const int part = (int)(t % sp);
  const int64_t vq = t / sp;
  const int64_t v = vq / n_groups, q = vq % n_groups;
  const int per = (L + sp - 1) / sp;
  const int j0 = part * per, j1 = j0 + per < L ? j0 + per : L;
  const G2A *T = reinterpret_cast<const G2A *>(T_aff) + q * L * kT;
  const uint32_t *w = ab + 2 * (v * m + q * L);
  G2J acc = G2J::inf();
  for (int win = 15; win >= 0; win--) {
    if (win != 15) {
      acc = jdbl(acc);
      acc = jdbl(acc);
    }
    for (int j = j0; j < j1; j++) {
      const uint32_t e = ((w[2 * j] >> (2 * win)) & 3u) + 4u * ((w[2 * j + 1] >> (2 * win)) & 3u);
      if (e) acc = jadd_mixed(acc, T[j * kT + e - 1]);
    }
  }
  at<G2J>(P_jac, t) = acc;
}

DX_HD void u_joint_reduce_one(const uint32_t *P_jac, uint32_t *U_aff, int64_t n_groups, int sp, int64_t pad,
                              const int64_t *pos, int64_t vq) {
  const int64_t v = vq / n_groups, q = vq % n_groups;
  G2J acc = at<G2J>(P_jac, vq * sp);
  for (int p = 1; p < sp; p++) acc = jadd(acc, at<G2J>(P_jac, vq * sp + p));
  at<G2A>(U_aff, pos ? pos[vq] : v * pad + q) = to_affine(acc);
}

DX_HD void slice_sum_one(const uint32_t *src, const int32_t *idx, const int64_t *start, const int32_t *len,
                         uint32_t *out, int src_aff, int64_t idx_mod, int64_t s) {
  const int64_t b = start[s];
  const int n = len[s];
  G2J acc = G2J::inf();
  for (int k = 0; k < n; k++) {
    int64_t e = idx ? idx[b + k] : b + k;
    if (idx_mod > 0) e %= idx_mod;
    if (src_aff)
      acc = jadd_mixed(acc, at<G2A>(src, e));
    else
      acc = jadd(acc, at<G2J>(src, e));
  }
  at<G2J>(out, s) = acc;
}

DX_HD void mul_small_one(const uint32_t *in_jac, const int32_t *d, uint32_t *out, int64_t i) {
  const G2J p = at<G2J>(in_jac, i);
  const uint32_t k = (uint32_t)d[i];
  G2J r = G2J::inf();
  for (int bit = 30; bit >= 0; bit--) {
    r = jdbl(r);
    if ((k >> bit) & 1u) r = jadd(r, p);
  }
  at<G2J>(out, i) = r;
}

DX_HD void horner_one(const uint32_t *S_jac, uint32_t *out_aff, int W, int c, int64_t stride, int64_t offset,
                      int64_t g) {
  G2J acc = at<G2J>(S_jac, g * W + W - 1);
  for (int w = W - 2; w >= 0; w--) {
    for (int k = 0; k < c; k++) acc = jdbl(acc);
    acc = jadd(acc, at<G2J>(S_jac, g * W + w));
  }
  at<G2A>(out_aff, g * stride + offset) = to_affine(acc);
}

DX_HD void msm_uv_one(const uint32_t *Y_jac, uint32_t *UV, int64_t n_groups, int64_t pad, int64_t t) {
  const int64_t v = t / (n_groups + 1), q = t % (n_groups + 1);
  G1A a;
  if (q < n_groups) {
    G1J y = at<G1J>(Y_jac, q);
    y.y = fneg(y.y);
    a = to_affine(y);
  } else {
    a = g1_generator();
  }
  if (a.is_inf()) {
    at<G1A>(UV, v * pad + q) = G1A::inf();
    return;
  }
  const Fp iy = finv(a.y);
  at<G1A>(UV, v * pad + q) = G1A{fmul(a.x, iy), iy};
}

// Bucket keys of a c-bit-window Pippenger plan: entry (t, w) of the n x W
// grid gets key ((g_t W + w) << c) | d_tw and item t, or the sentinel key
// 0x7fffffff (sorted past every bucket) when its digit d_tw is zero.
DX_HD void msm_keys_one(const uint32_t *k, const int32_t *grp, int64_t gstride, int c, int W, int32_t *keys,
                        int32_t *items, int64_t e) {
  const int64_t t = e / W;
  const int w = (int)(e % W);
  const uint32_t *kt = k + 8 * t;
  const int bit = w * c, li = bit >> 5, sh = bit & 31;
  uint32_t d = li < 8 ? kt[li] >> sh : 0u;
  if (sh + c > 32 && li + 1 < 8) d |= kt[li + 1] << (32 - sh);
  d &= (1u << c) - 1u;
  const int64_t g = grp ? grp[t] : (gstride > 0 ? t / gstride : 0);  // group of entry t: explicit or t / gstride
  keys[e] = d ? (int32_t)((((int64_t)g * W + w) << c) | d) : 0x7fffffff;
  items[e] = (int32_t)t;
}

#define DX_TID() const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x
// Bucket weights of a Pippenger window by running sums, per chunk of
// buckets whose digits lie in one aligned range [base, base + L): with the
// buckets sorted by digit, sum_i d_i B_i = base * sum_i B_i + sum_t A_t,
// A_t = sum_{d_i - base >= t} B_i for t = top .. 1 -- about 2 additions per
// bucket plus one short multiplication by base per chunk, instead of one
// double-and-add by a c-bit digit per bucket (~20 G2 operations each).
DX_HD void chunk_weight_one(const uint32_t *B_jac, const int32_t *d, const int64_t *start, const int32_t *len,
                            const int32_t *base, uint32_t *out, int64_t ch) {
  const int64_t a = start[ch];
  const int n = len[ch];
  const uint32_t b0 = (uint32_t)base[ch];
  G2J acc = G2J::inf(), tot = G2J::inf();
  int i = n - 1;
  int t = (int)((uint32_t)d[a + i] - b0);
  for (; t >= 1; t--) {
    while (i >= 0 && (int)((uint32_t)d[a + i] - b0) == t) {
      acc = jadd(acc, at<G2J>(B_jac, a + i));
      i--;
    }
    tot = jadd(tot, acc);
  }
  for (; i >= 0; i--) acc = jadd(acc, at<G2J>(B_jac, a + i));  // offset 0: weight base only
  if (b0) {  // base * acc, double-and-add from the base's top bit
    G2J m = acc;
    for (int bit = 30 - __builtin_clz(b0); bit >= 0; bit--) {
      m = jdbl(m);
      if ((b0 >> bit) & 1u) m = jadd(m, acc);
    }
    tot = jadd(tot, m);
  }
  at<G2J>(out, ch) = tot;
}

__global__ void __launch_bounds__(256) msm_keys_kernel(const uint32_t *k, const int32_t *grp, int64_t gstride,
                                                       int64_t n, int c, int W, int32_t *keys, int32_t *items) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n * W) msm_keys_one(k, grp, gstride, c, W, keys, items, i);
}
__global__ void __launch_bounds__(kWG) DX_OCC joint_table_kernel(const uint32_t *V, uint32_t *T, int64_t m) {
  DX_TID();
  if (i < m) joint_table_one(V, T, i);
}
__global__ void __launch_bounds__(kWG) DX_OCC u_joint_kernel(const uint32_t *T, const uint32_t *ab, uint32_t *U,
                                                            int64_t n_groups, int L, int64_t pad, const int64_t *pos,
                                                            int64_t n) {
  DX_TID();
  if (i < n) u_joint_one(T, ab, U, n_groups, L, pad, pos, i);
}
__global__ void __launch_bounds__(kWG) DX_OCC u_joint_reduce_kernel(const uint32_t *P, uint32_t *U, int64_t n_groups,
                                                                   int sp, int64_t pad, const int64_t *pos,
                                                                   int64_t n) {
  DX_TID();
  if (i < n) u_joint_reduce_one(P, U, n_groups, sp, pad, pos, i);
}
__global__ void __launch_bounds__(kWG) DX_OCC u_joint_part_kernel(const uint32_t *T, const uint32_t *ab,
                                                                 uint32_t *P, int64_t n_groups, int L, int sp,
                                                                 int64_t n) {
  DX_TID();
  if (i < n) u_joint_part_one(T, ab, P, n_groups, L, sp, i);
}
// The split combination with its reduction in the same workgroup: the sp
// lanes of a (v, q) are adjacent (sp | 64), add their partials pairwise
// through LDS (log2 sp rounds) and the first normalises -- no Jacobian
// partials through HBM and no second, one-lane-per-(v, q) launch (a pool
// part's ~23k (v, q) filled a third of the SIMDs there, 2.4 ms of the U chain,
// profiles/r6/prof/timeline_part6.txt).  Every lane reaches every barrier.
__global__ void __launch_bounds__(kWG) DX_OCC u_joint_fused_kernel(const uint32_t *T, const uint32_t *ab, uint32_t *U,
                                                                  int64_t n_groups, int L, int sp, int64_t pad,
                                                                  const int64_t *pos, int64_t n) {
  __shared__ G2J red[kWG];
  DX_TID();
  const bool live = i < n * sp;
  G2J acc = G2J::inf();
  if (live) {
    const int part = (int)(i % sp);
    const int64_t vq = i / sp;
    const int64_t v = vq / n_groups, q = vq % n_groups;
    const int64_t m = n_groups * L;
    const int per = (L + sp - 1) / sp;
    const int j0 = part * per, j1 = j0 + per < L ? j0 + per : L;
    const G2A *Tq = reinterpret_cast<const G2A *>(T) + q * L * kT;
    const uint32_t *w = ab + 2 * (v * m + q * L);
    for (int win = 15; win >= 0; win--) {
      if (win != 15) {
        acc = jdbl(acc);
        acc = jdbl(acc);
      }
      for (int j = j0; j < j1; j++) {
        const uint32_t e = ((w[2 * j] >> (2 * win)) & 3u) + 4u * ((w[2 * j + 1] >> (2 * win)) & 3u);
        if (e) acc = jadd_mixed(acc, Tq[j * kT + e - 1]);
      }
    }
  }
  const int part = (int)(threadIdx.x % sp);
  for (int st = 1; st < sp; st <<= 1) {
    if (part % (2 * st) == st) red[threadIdx.x] = acc;
    __syncthreads();
    if (part % (2 * st) == 0) acc = jadd(acc, red[threadIdx.x + st]);
    __syncthreads();
  }
  if (live && part == 0) {
    const int64_t vq = i / sp;
    const int64_t v = vq / n_groups, q = vq % n_groups;
    at<G2A>(U, pos ? pos[vq] : v * pad + q) = to_affine(acc);
  }
}
__global__ void __launch_bounds__(kWG) DX_OCC slice_sum_kernel(const uint32_t *src, const int32_t *idx,
                                                              const int64_t *start, const int32_t *len,
                                                              uint32_t *out, int src_aff, int64_t idx_mod,
                                                              int64_t n) {
  DX_TID();
  if (i < n) slice_sum_one(src, idx, start, len, out, src_aff, idx_mod, i);
}
__global__ void __launch_bounds__(kWG) DX_OCC mul_small_kernel(const uint32_t *in, const int32_t *d, uint32_t *out,
                                                              int64_t n) {
  DX_TID();
  if (i < n) mul_small_one(in, d, out, i);
}
__global__ void __launch_bounds__(kWG) DX_OCC chunk_weight_kernel(const uint32_t *B, const int32_t *d,
                                                                 const int64_t *start, const int32_t *len,
                                                                 const int32_t *base, uint32_t *out, int64_t n) {
  DX_TID();
  if (i < n) chunk_weight_one(B, d, start, len, base, out, i);
}
__global__ void __launch_bounds__(kWG) DX_OCC horner_kernel(const uint32_t *S, uint32_t *out, int W, int c,
                                                           int64_t stride, int64_t offset, int64_t n) {
  DX_TID();
  if (i < n) horner_one(S, out, W, c, stride, offset, i);
}
__global__ void __launch_bounds__(kWG) DX_OCC msm_uv_kernel(const uint32_t *Y, uint32_t *UV, int64_t n_groups,
                                                           int64_t pad, int64_t n) {
  DX_TID();
  if (i < n) msm_uv_one(Y, UV, n_groups, pad, i);
}
#undef DX_TID

inline dim3 grid_of(int64_t n) { return dim3((unsigned)((n + kWG - 1) / kWG)); }
}  // namespace

extern "C" {

// grp: group per scalar, or nullptr and gstride > 0 (group = t / gstride), or neither (one group)
int dx_msm_keys(int on_gpu, void *stream, const uint32_t *k, const int32_t *grp, int64_t gstride, int64_t n, int c,
                int W, int32_t *keys, int32_t *items) {
  if (n <= 0) return 0;
  if (!on_gpu) {
    host_for_each(n * W, [=](int64_t e) { msm_keys_one(k, grp, gstride, c, W, keys, items, e); });
    return 0;
  }
  hipLaunchKernelGGL(msm_keys_kernel, dim3((unsigned)((n * W + 255) / 256)), dim3(256), 0, (hipStream_t)stream, k,
                     grp, gstride, n, c, W, keys, items);
  return check_hip(hipGetLastError(), "msm_keys");
}

int dx_g2_joint_table(int on_gpu, void *stream, const uint32_t *V_aff, uint32_t *T_aff, int64_t m) {
  if (m <= 0) return 0;
  if (!on_gpu) {
    host_for_each(m, [=](int64_t it) { joint_table_one(V_aff, T_aff, it); });
    return 0;
  }
  hipLaunchKernelGGL(joint_table_kernel, grid_of(m), dim3(kWG), 0, (hipStream_t)stream, V_aff, T_aff, m);
  return check_hip(hipGetLastError(), "g2_joint_table");
}

// U[v*pad + q] = affine(sum_{j<L} (a + b lambda)_{v, q*L+j} V_{q*L+j}) for
// v < G, q < n_groups; ab [G*m, 2] (m = n_groups * L) are the 32-bit halves.
int dx_rp_u_joint(int on_gpu, void *stream, const uint32_t *T_aff, const uint32_t *ab, uint32_t *U_aff,
                  int64_t n_groups, int G, int L, int64_t pad, const int64_t *pos) {
  const int64_t n = (int64_t)G * n_groups;
  if (n <= 0) return 0;
  if (!on_gpu) {
    host_for_each(n, [=](int64_t t) { u_joint_one(T_aff, ab, U_aff, n_groups, L, pad, pos, t); });
    return 0;
  }
  hipLaunchKernelGGL(u_joint_kernel, grid_of(n), dim3(kWG), 0, (hipStream_t)stream, T_aff, ab, U_aff, n_groups, L,
                     pad, pos, n);
  return check_hip(hipGetLastError(), "rp_u_joint");
}

// dx_rp_u_joint with each (v, q) split over sp threads (tmp: G * n_groups * sp Jacobian rows)
int dx_rp_u_joint_split(int on_gpu, void *stream, const uint32_t *T_aff, const uint32_t *ab, uint32_t *U_aff,
                        int64_t n_groups, int G, int L, int64_t pad, int sp, uint32_t *tmp, const int64_t *pos) {
  const int64_t n = (int64_t)G * n_groups;
  if (n <= 0) return 0;
  if (!on_gpu) {
    host_for_each(n * sp, [=](int64_t t) { u_joint_part_one(T_aff, ab, tmp, n_groups, L, sp, t); });
    host_for_each(n, [=](int64_t t) { u_joint_reduce_one(tmp, U_aff, n_groups, sp, pad, pos, t); });
    return 0;
  }
  if (kWG % sp == 0) {
    hipLaunchKernelGGL(u_joint_fused_kernel, grid_of(n * sp), dim3(kWG), 0, (hipStream_t)stream, T_aff, ab, U_aff,
                       n_groups, L, sp, pad, pos, n);
    return check_hip(hipGetLastError(), "rp_u_joint_fused");
  }
  hipLaunchKernelGGL(u_joint_part_kernel, grid_of(n * sp), dim3(kWG), 0, (hipStream_t)stream, T_aff, ab, tmp,
                     n_groups, L, sp, n * sp);
  hipLaunchKernelGGL(u_joint_reduce_kernel, grid_of(n), dim3(kWG), 0, (hipStream_t)stream, tmp, U_aff, n_groups, sp,
                     pad, pos, n);
  return check_hip(hipGetLastError(), "rp_u_joint_split");
}

// out[s] = sum_{k < len[s]} src[e_k], e_k = idx[start[s] + k] (mod idx_mod when
// > 0) or start[s] + k; src affine G2 (mixed additions) or Jacobian G2.
int dx_g2_slice_sum(int on_gpu, void *stream, const uint32_t *src, const int32_t *idx, const int64_t *start,
                    const int32_t *len, uint32_t *out, int64_t n_slices, int src_aff, int64_t idx_mod) {
  if (n_slices <= 0) return 0;
  if (!on_gpu) {
    host_for_each(n_slices, [=](int64_t s) { slice_sum_one(src, idx, start, len, out, src_aff, idx_mod, s); });
    return 0;
  }
  hipLaunchKernelGGL(slice_sum_kernel, grid_of(n_slices), dim3(kWG), 0, (hipStream_t)stream, src, idx, start, len,
                     out, src_aff, idx_mod, n_slices);
  return check_hip(hipGetLastError(), "g2_slice_sum");
}

// out[i] = d[i] * in[i] (Jacobian), 0 <= d[i] < 2^31: the Pippenger bucket weights
int dx_g2_mul_small(int on_gpu, void *stream, const uint32_t *in_jac, const int32_t *d, uint32_t *out, int64_t n) {
  if (n <= 0) return 0;
  if (!on_gpu) {
    host_for_each(n, [=](int64_t i) { mul_small_one(in_jac, d, out, i); });
    return 0;
  }
  hipLaunchKernelGGL(mul_small_kernel, grid_of(n), dim3(kWG), 0, (hipStream_t)stream, in_jac, d, out, n);
  return check_hip(hipGetLastError(), "g2_mul_small");
}

// out[ch] = sum_{i in chunk ch} d[i] * B[i] (Jacobian; chunk = start/len over
// digit-sorted buckets whose digits lie in [base, base + L))
int dx_g2_chunk_weight(int on_gpu, void *stream, const uint32_t *B_jac, const int32_t *d, const int64_t *start,
                       const int32_t *len, const int32_t *base, uint32_t *out, int64_t n) {
  if (n <= 0) return 0;
  if (!on_gpu) {
    host_for_each(n, [=](int64_t i) { chunk_weight_one(B_jac, d, start, len, base, out, i); });
    return 0;
  }
  hipLaunchKernelGGL(chunk_weight_kernel, grid_of(n), dim3(kWG), 0, (hipStream_t)stream, B_jac, d, start, len, base,
                     out, n);
  return check_hip(hipGetLastError(), "g2_chunk_weight");
}

// Per group g < G: acc = S[g*W + W-1]; acc = 2^c acc + S[g*W + w] for w = W-2..0;
// out_aff[g*stride + offset] = affine(acc).  One lane per group (W*c
// doublings): the MSM result lands in the pairing input list on the device.
int dx_g2_horner(int on_gpu, void *stream, const uint32_t *S_jac, uint32_t *out_aff, int G, int W, int c,
                 int64_t stride, int64_t offset) {
  if (G <= 0) return 0;
  if (!on_gpu) {
    host_for_each(G, [=](int64_t g) { horner_one(S_jac, out_aff, W, c, stride, offset, g); }, 2);
    return 0;
  }
  hipLaunchKernelGGL(horner_kernel, grid_of(G), dim3(kWG), 0, (hipStream_t)stream, S_jac, out_aff, W, c, stride,
                     offset, (int64_t)G);
  return check_hip(hipGetLastError(), "g2_horner");
}

// The G1 side of the regrouped fold in the normalised (u, v) = (x/y, 1/y)
// form: UV[v*pad + q] = uv(-Y_q) for q < n_groups and UV[v*pad + n_groups] =
// uv(B), for every verifier v < G (rows left untouched stay infinity).
int dx_rp_msm_uv(int on_gpu, void *stream, const uint32_t *Y_jac, uint32_t *UV, int64_t n_groups, int G,
                 int64_t pad) {
  const int64_t n = (int64_t)G * (n_groups + 1);
  if (n <= 0) return 0;
  if (!on_gpu) {
    host_for_each(n, [=](int64_t t) { msm_uv_one(Y_jac, UV, n_groups, pad, t); });
    return 0;
  }
  hipLaunchKernelGGL(msm_uv_kernel, grid_of(n), dim3(kWG), 0, (hipStream_t)stream, Y_jac, UV, n_groups, pad, n);
  return check_hip(hipGetLastError(), "rp_msm_uv");
}

}  // extern "C"
