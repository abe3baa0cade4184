// Pairing / GT batch ops (K7, K8): kyber bn256 Pair + GT arithmetic used by
// lib/range/range_proof.go:396-397 (prove) and :540-546 (verify).
// C ABI consumed by drynx_amd/native (ctypes).  Every entry point takes
// (on_gpu, stream): on_gpu launches a gfx950 kernel on that HIP stream (torch's
// current stream), otherwise the same functor runs on the host thread pool.
#include "common.h"

extern "C" {
// ---------------------------------------------------------------- pairing / GT
int dx_miller_loop(int on_gpu, void *stream, const uint32_t *P_aff, const uint32_t *Q_aff, uint32_t *out, int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) { at<Fp12>(out, i) = miller_loop(at<G1A>(P_aff, i), at<G2A>(Q_aff, i)); };
  return run(on_gpu, stream, n, op, true, "miller_loop");
}

int dx_final_exp(int on_gpu, void *stream, const uint32_t *in, uint32_t *out, int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) { at<Fp12>(out, i) = final_exp(at<Fp12>(in, i)); };
  return run(on_gpu, stream, n, op, true, "final_exp");
}

int dx_pairing(int on_gpu, void *stream, const uint32_t *P_aff, const uint32_t *Q_aff, uint32_t *out, int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) { at<Fp12>(out, i) = pairing(at<G1A>(P_aff, i), at<G2A>(Q_aff, i)); };
  return run(on_gpu, stream, n, op, true, "pairing");
}

int dx_gt_mul(int on_gpu, void *stream, const uint32_t *a, const uint32_t *b, uint32_t *out, int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) { at<Fp12>(out, i) = mul(at<Fp12>(a, i), at<Fp12>(b, i)); };
  return run(on_gpu, stream, n, op, true, "gt_mul");
}

// out_i = a_i^-1 in Fp12* (any non-zero element, not only the cyclotomic
// subgroup where the conjugate is the inverse)
int dx_gt_inv(int on_gpu, void *stream, const uint32_t *a, uint32_t *out, int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) { at<Fp12>(out, i) = inv(at<Fp12>(a, i)); };
  return run(on_gpu, stream, n, op, true, "gt_inv");
}

int dx_gt_pow(int on_gpu, void *stream, const uint32_t *a, const uint32_t *scalars, uint32_t *out, int64_t n,
              int a_bcast) {
  auto op = [=] __host__ __device__(int64_t i) {
    at<Fp12>(out, i) = gt_pow(at<Fp12>(a, a_bcast ? 0 : i), scalars + 8 * i);
  };
  return run(on_gpu, stream, n, op, true, "gt_pow");
}

int dx_gt_eq(int on_gpu, void *stream, const uint32_t *a, const uint32_t *b, uint8_t *out, int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) { out[i] = at<Fp12>(a, i) == at<Fp12>(b, i) ? 1 : 0; };
  return run(on_gpu, stream, n, op, false, "gt_eq");
}

// comb table for fixed-base GT exponentiation (32 x 256 entries of Fp12)
// Two-phase comb table in GT: 256 cyclotomic squarings per base, then <= 7
// Fp12 products per entry.
int dx_gt_fb_table(int on_gpu, void *stream, const uint32_t *base, uint32_t *work, uint32_t *table, int64_t n_bases) {
  auto p1 = [=] __host__ __device__(int64_t b) {
    Fp12 acc = at<Fp12>(base, b);
    for (int k = 0; k < 256; k++) {
      at<Fp12>(work, b * 256 + k) = acc;
      acc = cyclotomic_sqr(acc);
    }
  };
  int rc = run(on_gpu, stream, n_bases, p1, true, "gt_fb_table_pow2");
  if (rc) return rc;
  auto p2 = [=] __host__ __device__(int64_t t) {
    int64_t b = t / 8192, i = t % 8192;
    int w = (int)(i >> 8), d = (int)(i & 255);
    Fp12 acc = Fp12::one();
    for (int bit = 0; bit < 8; bit++)
      if ((d >> bit) & 1) acc = mul(acc, at<Fp12>(work, b * 256 + 8 * w + bit));
    at<Fp12>(table, t) = acc;
  };
  return run(on_gpu, stream, n_bases * 8192, p2, true, "gt_fb_table");
}

int dx_gt_fb_pow(int on_gpu, void *stream, const uint32_t *tables, const int32_t *tab_idx, const uint32_t *scalars,
                 uint32_t *out, int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) {
    const Fp12 *T = reinterpret_cast<const Fp12 *>(tables) + (int64_t)(tab_idx ? tab_idx[i] : 0) * 8192;
    at<Fp12>(out, i) = gt_fixed_pow(T, scalars + 8 * i);
  };
  return run(on_gpu, stream, n, op, true, "gt_fb_pow");
}

// 4-bit comb tables (gt_fixed_pow4 layout): work[b*64 + w] = base^(16^w), then
// table[b*960 + w*15 + d - 1] = base^(d * 16^w).
int dx_gt_fb4_table(int on_gpu, void *stream, const uint32_t *base, uint32_t *work, uint32_t *table,
                    int64_t n_bases) {
  auto p1 = [=] __host__ __device__(int64_t b) {
    Fp12 acc = at<Fp12>(base, b);
    for (int w = 0; w < 64; w++) {
      at<Fp12>(work, b * 64 + w) = acc;
      acc = cyclotomic_sqr(cyclotomic_sqr(cyclotomic_sqr(cyclotomic_sqr(acc))));
    }
  };
  int rc = run(on_gpu, stream, n_bases, p1, true, "gt_fb4_table_pow16");
  if (rc) return rc;
  auto p2 = [=] __host__ __device__(int64_t t) {
    const int64_t b = t / 960, i = t % 960;
    const int w = (int)(i / 15), d = (int)(i % 15) + 1;
    Fp12 q = at<Fp12>(work, b * 64 + w), acc = Fp12::one();
    for (int bit = 0; bit < 4; bit++) {
      if ((d >> bit) & 1) acc = mul(acc, q);
      if (bit < 3 && (d >> (bit + 1))) q = cyclotomic_sqr(q);
    }
    at<Fp12>(table, t) = acc;
  };
  return run(on_gpu, stream, n_bases * 960, p2, true, "gt_fb4_table");
}

int dx_gt_fb4_pow(int on_gpu, void *stream, const uint32_t *tables, const int32_t *tab_idx, const uint32_t *scalars,
                  uint32_t *out, int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) {
    const Fp12 *T = reinterpret_cast<const Fp12 *>(tables) + (int64_t)(tab_idx ? tab_idx[i] : 0) * 960;
    at<Fp12>(out, i) = gt_fixed_pow4(T, scalars + 8 * i);
  };
  return run(on_gpu, stream, n, op, true, "gt_fb4_pow");
}

// dx_gt_cyclotomic (a_ij in the cyclotomic subgroup): csrc/kernels/dx_check_inl.hip

// Exact membership of the prime-order GT for elements of the cyclotomic
// subgroup: p = 6u^2 (mod r), so x^r = 1 iff x^p == x^(6u^2).  x^p is ONE
// Frobenius map; x^(6u^2) = ((x^u)^u)^6 two cyclotomic u-ladders (62
// Granger-Scott squarings each) and three products -- instead of two generic
// 254/127-bit exponentiations.  The caller guarantees cyclotomic inputs.
int dx_gt_membership(int on_gpu, void *stream, const uint32_t *a, uint8_t *out, int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) {
    const Fp12 x = at<Fp12>(a, i);
    const Fp12 y = cyc_pow_u(cyc_pow_u(x));
    const Fp12 y2 = cyclotomic_sqr(y);
    out[i] = frob<1>(x) == mul(y2, cyclotomic_sqr(y2)) ? 1 : 0;
  };
  return run(on_gpu, stream, n, op, true, "gt_membership");
}

// product over axis 0 chunks of in[n_items][n_groups] Fp12 (same scheme as g1_sum_chunks)
int dx_gt_prod_chunks(int on_gpu, void *stream, const uint32_t *in, uint32_t *out, int64_t n_items, int64_t n_groups,
                      int64_t chunk) {
  int64_t n_chunks = (n_items + chunk - 1) / chunk;
  auto op = [=] __host__ __device__(int64_t t) {
    int64_t c = t / n_groups, g = t % n_groups;
    int64_t s = c * chunk, e = s + chunk < n_items ? s + chunk : n_items;
    Fp12 acc = Fp12::one();
    for (int64_t i = s; i < e; i++) acc = mul(acc, at<Fp12>(in, i * n_groups + g));
    at<Fp12>(out, t) = acc;
  };
  return run(on_gpu, stream, n_chunks * n_groups, op, true, "gt_prod_chunks");
}


}  // extern "C"
