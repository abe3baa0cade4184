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

namespace {
// psi on Jacobian coordinates: (X, Y, Z) -> (conj(X) twx, conj(Y) twy, conj(Z)).
DX_HD G2J psi_jac(const G2J &q) {
  return {mul(conj(q.x), Fp2::from_limbs(Frob::TWX1)), mul(conj(q.y), Fp2::from_limbs(Frob::TWY1)), conj(q.z)};
}
}  // namespace

extern "C" {
// G2 membership of a twist point (range-proof V_ij): on the curve and
//   [u+1] Q + psi([u] Q) + psi^2([u] Q) == psi^3([2u] Q)
// (the BN-curve test of Dai-Lin-Zhao-Zhou 2022: one 63-bit ladder [u] Q instead
// of the 127-bit [6u^2] Q of psi(Q) == [6u^2] Q).  Exact: the cofactor 2p - r is
// squarefree (10069 * 5864401 * 1875725156269 * p54), psi acts on each cyclic
// prime-order part as a scalar, and the test's endomorphism is non-zero on each
// (tests/test_range_hardening.py checks a point of every torsion order).
int dx_g2_subgroup(int on_gpu, void *stream, const uint32_t *aff, uint8_t *out, int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) {
    const G2A q = at<G2A>(aff, i);
    if (!on_curve(q)) {
      out[i] = 0;
      return;
    }
    if (q.is_inf()) {
      out[i] = 1;
      return;
    }
    G2J uq = G2J::from_aff(q);  // top bit of u (bit 62)
    for (int b = 61; b >= 0; --b) {
      uq = jdbl(uq);
      if ((BN_U >> b) & 1ull) uq = jadd_mixed(uq, q);
    }
    const G2J p1 = psi_jac(uq);
    const G2J lhs = jadd(jadd(jadd_mixed(uq, q), p1), psi_jac(p1));
    const G2J rhs = psi_jac(psi_jac(psi_jac(jdbl(uq))));
    out[i] = jeq(lhs, rhs) ? 1 : 0;
  };
  return run(on_gpu, stream, n, op, true, "g2_subgroup");
}

int dx_g2_on_curve(int on_gpu, void *stream, const uint32_t *aff, uint8_t *out, int64_t n) {
  auto op = [=] __host__ __device__(int64_t i) { out[i] = on_curve(at<G2A>(aff, i)) ? 1 : 0; };
  return run(on_gpu, stream, n, op, false, "g2_on_curve");
}

}  // extern "C"
