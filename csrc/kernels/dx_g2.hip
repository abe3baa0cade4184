// G2 batch ops (K6): BB-signature setup and range-proof V_ij = v_ij * A_{i,phi_j}
// (lib/range/range_proof.go:259-288,392).
// C ABI consumed by drynx_amd/native (ctypes).  Every entry point takes
// (on_gpu, stream): on_gpu launches a gfx950 kernel on that HIP stream (torch's
// current stream), otherwise the same functor runs on the host thread pool.
#include "common.h"

extern "C" {
// ---------------------------------------------------------------- G2
// Same two-phase comb-table build as dx_g1_fb_table, over the twist.
int dx_g2_fb_table(int on_gpu, void *stream, const uint32_t *bases_aff, uint32_t *work, uint32_t *table,
                   int64_t n_bases) {
  auto p1 = [=] __host__ __device__(int64_t b) {
    G2J acc = G2J::from_aff(at<G2A>(bases_aff, b));
    for (int k = 0; k < 256; k++) {
      at<G2J>(work, b * 256 + k) = acc;
      acc = jdbl(acc);
    }
  };
  int rc = run(on_gpu, stream, n_bases, p1, true, "g2_fb_table_pow2");
  if (rc) return rc;
  auto p2 = [=] __host__ __device__(int64_t t) {
    int64_t b = t / 8192, i = t % 8192;
    int w = (int)(i >> 8), d = (int)(i & 255);
    G2J acc = G2J::inf();
    for (int bit = 0; bit < 8; bit++)
      if ((d >> bit) & 1) acc = jadd(acc, at<G2J>(work, b * 256 + 8 * w + bit));
    at<G2A>(table, t) = to_affine(acc);
  };
  return run(on_gpu, stream, n_bases * 8192, p2, true, "g2_fb_table");
}

// out[i] = k[i] * base, table chosen per item from tables[tab_idx[i]] (tab_idx may be null -> table 0)
int dx_g2_fb_mul(int on_gpu, void *stream, const uint32_t *tables, const int32_t *tab_idx, const uint32_t *scalars,
                 uint32_t *out_aff, int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) {
    const G2A *T = reinterpret_cast<const G2A *>(tables) + (int64_t)(tab_idx ? tab_idx[i] : 0) * 8192;
    at<G2A>(out_aff, i) = to_affine(fixed_base_mul(T, scalars + 8 * i));
  };
  return run(on_gpu, stream, n, op, true, "g2_fb_mul");
}

// 4-bit comb tables (fixed_base_mul4 layout): work[b*64 + w] = 16^w * base
// (Jacobian), then table[b*960 + w*15 + d - 1] = d * 16^w * base (affine).
int dx_g2_fb4_table(int on_gpu, void *stream, const uint32_t *bases_aff, uint32_t *work, uint32_t *table,
                    int64_t n_bases) {
  auto p1 = [=] __host__ __device__(int64_t b) {
    G2J acc = G2J::from_aff(at<G2A>(bases_aff, b));
    for (int w = 0; w < 64; w++) {
      at<G2J>(work, b * 64 + w) = acc;
      acc = jdbl(jdbl(jdbl(jdbl(acc))));
    }
  };
  int rc = run(on_gpu, stream, n_bases, p1, true, "g2_fb4_table_pow16");
  if (rc) return rc;
  auto p2 = [=] __host__ __device__(int64_t t) {
    const int64_t b = t / 960, i = t % 960;
    const int w = (int)(i / 15), d = (int)(i % 15) + 1;
    G2J q = at<G2J>(work, b * 64 + w), acc = G2J::inf();
    for (int bit = 0; bit < 4; bit++) {
      if ((d >> bit) & 1) acc = jadd(acc, q);
      if (bit < 3 && (d >> (bit + 1))) q = jdbl(q);
    }
    at<G2A>(table, t) = to_affine(acc);
  };
  return run(on_gpu, stream, n_bases * 960, p2, true, "g2_fb4_table");
}

int dx_g2_fb4_mul(int on_gpu, void *stream, const uint32_t *tables, const int32_t *tab_idx, const uint32_t *scalars,
                  uint32_t *out_aff, int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) {
    const G2A *T = reinterpret_cast<const G2A *>(tables) + (int64_t)(tab_idx ? tab_idx[i] : 0) * 960;
    at<G2A>(out_aff, i) = to_affine(fixed_base_mul4(T, scalars + 8 * i));
  };
  return run(on_gpu, stream, n, op, true, "g2_fb4_mul");
}

int dx_g2_mul(int on_gpu, void *stream, const uint32_t *pts_aff, const uint32_t *scalars, uint32_t *out_aff, int64_t n,
              int pt_bcast) {
  auto op = [=] __host__ __device__(int64_t i) {
    G2J p = G2J::from_aff(at<G2A>(pts_aff, pt_bcast ? 0 : i));
    at<G2A>(out_aff, i) = to_affine(scalar_mul(p, scalars + 8 * i));
  };
  return run(on_gpu, stream, n, op, true, "g2_mul");
}

}  // extern "C"

extern "C" {
// dx_g2_subgroup: csrc/kernels/dx_check_inl.hip (force-inlined, spill-free)
int dx_g2_on_curve(int on_gpu, void *stream, const uint32_t *aff, uint8_t *out, int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) { out[i] = on_curve(at<G2A>(aff, i)) ? 1 : 0; };
  return run(on_gpu, stream, n, op, false, "g2_on_curve");
}

}  // extern "C"
