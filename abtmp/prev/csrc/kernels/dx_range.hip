// Fused range-proof kernels (K15 prove, K16 batched verify).
//
// Reference: lib/range/range_proof.go.  Per value, digit j and server i the
// prover publishes a_ij = e(-s_j B, V_ij) * e(t_j B, B2) (:396-397) and the
// verifier checks a_ij == e(c y_i, V_ij) e(-Zphi_j B, V_ij) e(Zv_ij B, B2)
// (:540-546) — 2 + 3 full pairings per (i, j) in the reference.
//
// Here:
//   prove  : a_ij = FE(ML(-s_j B, V_ij)) * gT^{t_j}   (gT = e(B,B2) comb table)
//   verify : all (p,i,j) of a list are folded with random 64-bit weights rho:
//            FE(prod_pij ML(rho (Zphi_j B - c y_i), V_ij)) * prod_pij a_ij^rho
//            == gT^{sum rho Zv}: ONE final exponentiation for the whole list.  One Miller loop per (p,i,j)
//            instead of three pairings.
// Item index: it = (p * S + i) * L + j.
#include "common.h"
#include "../bn254/gt_coop.h"

extern "C" {

// a[it] = FE(ML(negsB[p*L+j], V[it])) * gT^{t[p*L+j]}
int dx_rp_prove_a(int on_gpu, void *stream, const uint32_t *negsB_aff, const uint32_t *V_aff, const uint32_t *t_sc,
                  const uint32_t *gt_table, uint32_t *a_out, int64_t n_items, int S, int L) {
  auto op = [=] __host__ __device__(int64_t it) {
    int64_t j = it % L;
    int64_t p = it / ((int64_t)S * L);
    int64_t pj = p * L + j;
    Fp12 f = final_exp(miller_loop(at<G1A>(negsB_aff, pj), at<G2A>(V_aff, it)));
    Fp12 g = gt_fixed_pow(reinterpret_cast<const Fp12 *>(gt_table), t_sc + 8 * pj);
    at<Fp12>(a_out, it) = mul(f, g);
  };
  return run(on_gpu, stream, n_items, op, true, "rp_prove_a");
}

// Table-driven prover (no pairing per item): a[it] = g_phi^{e[it]} * gT^{t[p*L+j]}
// with g_phi = e(B, A_phi) comb-tabled per distinct signature point
// (gphi_tables[tab_idx[it]]) and e = -s_j v_ij computed on the device.
// gT^{t_pj} is shared by the S servers of a digit: computed once per (p, j)
// (first pass, into a_out rows it = (p*S)*L + j) and reused by the others.
// wbits = 8: gphi tables in the 8-bit comb layout (8192 entries per point);
// wbits = 4: the 4-bit layout (960 entries per point, gt_fixed_pow4).
int dx_rp_prove_a_tab(int on_gpu, void *stream, const uint32_t *gphi_tables, const int32_t *tab_idx,
                      const uint32_t *e_sc, const uint32_t *t_sc, const uint32_t *gt_table, uint32_t *a_out,
                      int64_t n_items, int S, int L, int wbits) {
  const int64_t n_pj = n_items / S;
  auto p1 = [=] __host__ __device__(int64_t pj) {
    const int64_t p = pj / L, j = pj % L;
    at<Fp12>(a_out, p * S * L + j) = gt_fixed_pow(reinterpret_cast<const Fp12 *>(gt_table), t_sc + 8 * pj);
  };
  int rc = run(on_gpu, stream, n_pj, p1, true, "rp_prove_gt_t");
  if (rc) return rc;
  // servers i = S-1 .. 0 read the shared row before server 0 overwrites it: run
  // the i > 0 items first, then i == 0
  for (int pass = 0; pass < 2; pass++) {
    const int64_t per = pass == 0 ? (int64_t)(S - 1) * L : (int64_t)L;  // items per value in this pass
    if (per == 0) continue;
    const int64_t n = n_pj / L * per;
    auto p2 = [=] __host__ __device__(int64_t k) {
      const int64_t p = k / per, r = k % per;
      const int64_t i = pass == 0 ? 1 + r / L : 0, j = r % L;
      const int64_t it = (p * S + i) * L + j;
      const Fp12 *T = reinterpret_cast<const Fp12 *>(gphi_tables) + (int64_t)tab_idx[it] * (wbits == 4 ? 960 : 8192);
      Fp12 f = wbits == 4 ? gt_fixed_pow4(T, e_sc + 8 * it) : gt_fixed_pow(T, e_sc + 8 * it);
      at<Fp12>(a_out, it) = mul(f, at<Fp12>(a_out, p * S * L + j));
    };
    rc = run(on_gpu, stream, n, p2, true, "rp_prove_a_tab");
    if (rc) return rc;
  }
  return 0;
}

// f[it] = ML(rho (ZB[p*L+j] - Y[p*S+i]), V[it]),  g[it] = a[it]^rho
// (the final exponentiation applies to the Miller product only: a_ij is already in GT)
int dx_rp_verify_items(int on_gpu, void *stream, const uint32_t *ZB_jac, const uint32_t *Y_jac, const uint32_t *rho,
                       const uint32_t *V_aff, const uint32_t *a, uint32_t *f_out, uint32_t *g_out, int64_t n_items,
                       int S, int L) {
  auto op = [=] __host__ __device__(int64_t it) {
    int64_t j = it % L;
    int64_t pi = it / L;  // p*S + i
    int64_t p = pi / S;
    G1J T = jadd(at<G1J>(ZB_jac, p * L + j), jneg(at<G1J>(Y_jac, pi)));
    G1A P = to_affine(scalar_mul(T, rho + 8 * it));
    at<Fp12>(f_out, it) = miller_loop(P, at<G2A>(V_aff, it));
    at<Fp12>(g_out, it) = gt_pow(at<Fp12>(a, it), rho + 8 * it);
  };
  return run(on_gpu, stream, n_items, op, true, "rp_verify_items");
}

}  // extern "C"

// GPU-only fused Miller fold: every 64-lane workgroup computes the Miller
// values of 64 items and folds them with an LDS tree, writing one Fp12 per
// workgroup -- the [n_items] intermediate never reaches HBM.  The a^rho side
// of the batch equation is a separate bucket multi-exponentiation
// (dx_gt_slice_prod below + rp_verify_products in native/__init__.py), so this
// kernel carries only the Miller-loop state.
namespace {
constexpr int kVW = 64;
__global__ void __launch_bounds__(kVW) DX_OCC rp_verify_fold_kernel(const uint32_t *ZB_jac, const uint32_t *Y_jac,
                                                              const uint32_t *rho, const uint32_t *V_aff,
                                                              uint32_t *f_blk, int64_t n_items, int S, int L) {
  // 32 Fp12 of LDS (12 KiB): the upper half of the live lanes hands its value
  // down each level.  With 24 KiB (one slot per lane) the LDS capped a CU at 6
  // of these workgroups, so a 99392-item batch (1553 workgroups) left 17 for a
  // second, nearly empty round; at 12 KiB the register file (2 waves per SIMD,
  // 8 per CU) is the cap and the whole batch is resident at once.
  __shared__ Fp12 sf[kVW / 2];
  const int lane = threadIdx.x;
  const int64_t it = (int64_t)blockIdx.x * kVW + lane;
  Fp12 f = Fp12::one();
  if (it < n_items) {
    int64_t j = it % L;
    int64_t pi = it / L;
    int64_t p = pi / S;
    G1J T = jadd(at<G1J>(ZB_jac, p * L + j), jneg(at<G1J>(Y_jac, pi)));
    G1A P = to_affine(scalar_mul(T, rho + 8 * it));
    f = miller_loop(P, at<G2A>(V_aff, it));
  }
  for (int s = kVW / 2; s > 0; s >>= 1) {
    if (lane >= s && lane < 2 * s) sf[lane - s] = f;
    __syncthreads();
    if (lane < s) f = mul(f, sf[lane]);
    __syncthreads();
  }
  if (lane == 0) at<Fp12>(f_blk, blockIdx.x) = f;
}
}  // namespace

extern "C" int dx_rp_verify_fold(void *stream, const uint32_t *ZB_jac, const uint32_t *Y_jac, const uint32_t *rho,
                                 const uint32_t *V_aff, uint32_t *f_blk, int64_t n_items, int S, int L) {
  if (n_items <= 0) return 0;
  int64_t blocks = (n_items + kVW - 1) / kVW;
  hipLaunchKernelGGL(rp_verify_fold_kernel, dim3((unsigned)blocks), dim3(kVW), 0, (hipStream_t)stream, ZB_jac, Y_jac,
                     rho, V_aff, f_blk, n_items, S, L);
  return check_hip(hipGetLastError(), "rp_verify_fold");
}

// Segmented GT products (bucket accumulation of a multi-exponentiation):
//   out[s] = prod_{k < len[s]} src[idx ? idx[start[s] + k] : start[s] + k]
// GPU: three lanes per slice (gt_coop.h).
namespace {
__global__ void __launch_bounds__(64) DX_OCC gt_slice_prod_coop(const uint32_t *src, const int64_t *idx,
                                                               const int64_t *start, const int32_t *len,
                                                               uint32_t *out, int64_t n_slices) {
  const coop::Role R = coop::role();
  const int64_t s = (int64_t)blockIdx.x * coop::kTriples + R.g;
  if (R.g >= coop::kTriples || s >= n_slices) return;  // whole triples leave together
  const int64_t b = start[s];
  const int n = len[s];
  const Fp12 *F = reinterpret_cast<const Fp12 *>(src);
  Fp6 x = coop::one(R);
  for (int k = 0; k < n; k++) coop::mul(x, coop::load(&F[idx ? idx[b + k] : b + k], false, R), R);
  coop::store(&at<Fp12>(out, s), x, R);
}
}  // namespace

extern "C" int dx_gt_slice_prod(int on_gpu, void *stream, const uint32_t *src, const int64_t *idx,
                                const int64_t *start, const int32_t *len, uint32_t *out, int64_t n_slices) {
  if (n_slices <= 0) return 0;
  if (!on_gpu) {
    host_for_each(n_slices, [=](int64_t s) {
      const int64_t b = start[s];
      const int n = len[s];
      Fp12 acc = Fp12::one();
      for (int k = 0; k < n; k++) acc = mul(acc, at<Fp12>(src, idx ? idx[b + k] : b + k));
      at<Fp12>(out, s) = acc;
    });
    return 0;
  }
  const unsigned blocks = (unsigned)((n_slices + coop::kTriples - 1) / coop::kTriples);
  hipLaunchKernelGGL(gt_slice_prod_coop, dim3(blocks), dim3(64), 0, (hipStream_t)stream, src, idx, start, len, out,
                     n_slices);
  return check_hip(hipGetLastError(), "gt_slice_prod");
}

// Bucket weights of a GT multi-exponentiation window by running products,
// per chunk of buckets whose digits lie in one aligned range [base, base + L)
// (the multiplicative form of dx_rpmsm.hip chunk_weight_one): with the
// buckets sorted by digit, prod_i B_i^(d_i) = (prod_i B_i)^base * prod_t A_t,
// A_t = prod_(d_i - base >= t) B_i for t = top .. 1 -- two products per bucket
// plus one short power per chunk, instead of a d-th power of every bucket
// (~16 products for an 11-bit digit).  Three lanes per chunk (gt_coop.h).
namespace {
__global__ void __launch_bounds__(64) DX_OCC gt_chunk_weight_coop(const uint32_t *B, const int32_t *d,
                                                                 const int64_t *start, const int32_t *len,
                                                                 const int32_t *base, uint32_t *out,
                                                                 int64_t n_chunks) {
  const coop::Role R = coop::role();
  const int64_t ch = (int64_t)blockIdx.x * coop::kTriples + R.g;
  if (R.g >= coop::kTriples || ch >= n_chunks) return;  // whole triples leave together
  const Fp12 *F = reinterpret_cast<const Fp12 *>(B);
  const int64_t a = start[ch];
  const int n = len[ch];
  const uint32_t b0 = (uint32_t)base[ch];
  Fp6 acc = coop::one(R), tot = coop::one(R);
  int i = n - 1;
  for (int t = n > 0 ? (int)((uint32_t)d[a + i] - b0) : 0; t >= 1; t--) {
    while (i >= 0 && (int)((uint32_t)d[a + i] - b0) == t) {
      coop::mul(acc, coop::load(&F[a + i], false, R), R);
      i--;
    }
    coop::mul(tot, acc, R);
  }
  for (; i >= 0; i--) coop::mul(acc, coop::load(&F[a + i], false, R), R);  // offset 0: weight base only
  if (b0) {  // acc^base from the base's top bit
    Fp6 m = acc;
    for (int bit = 30 - __builtin_clz(b0); bit >= 0; bit--) {
      coop::mul(m, m, R);
      if ((b0 >> bit) & 1u) coop::mul(m, acc, R);
    }
    coop::mul(tot, m, R);
  }
  coop::store(&at<Fp12>(out, ch), tot, R);
}
}  // namespace

extern "C" int dx_gt_chunk_weight(int on_gpu, void *stream, const uint32_t *B, const int32_t *d,
                                  const int64_t *start, const int32_t *len, const int32_t *base, uint32_t *out,
                                  int64_t n_chunks) {
  if (n_chunks <= 0) return 0;
  if (!on_gpu) {
    host_for_each(n_chunks, [=](int64_t ch) {
      const int64_t a = start[ch];
      const int n = len[ch];
      const uint32_t b0 = (uint32_t)base[ch];
      Fp12 acc = Fp12::one(), tot = Fp12::one();
      int i = n - 1;
      for (int t = n > 0 ? (int)((uint32_t)d[a + i] - b0) : 0; t >= 1; t--) {
        while (i >= 0 && (int)((uint32_t)d[a + i] - b0) == t) acc = mul(acc, at<Fp12>(B, a + i--));
        tot = mul(tot, acc);
      }
      for (; i >= 0; i--) acc = mul(acc, at<Fp12>(B, a + i));
      if (b0) {
        Fp12 m = acc;
        for (int bit = 30 - __builtin_clz(b0); bit >= 0; bit--) {
          m = mul(m, m);
          if ((b0 >> bit) & 1u) m = mul(m, acc);
        }
        tot = mul(tot, m);
      }
      at<Fp12>(out, ch) = tot;
    });
    return 0;
  }
  const unsigned blocks = (unsigned)((n_chunks + coop::kTriples - 1) / coop::kTriples);
  hipLaunchKernelGGL(gt_chunk_weight_coop, dim3(blocks), dim3(64), 0, (hipStream_t)stream, B, d, start, len, base,
                     out, n_chunks);
  return check_hip(hipGetLastError(), "gt_chunk_weight");
}
