// GLS-2 fixed-base tables with SIGNED 8-bit windows (prover table mode 7;
// K6/K7 of the range-proof prover, lib/range/range_proof.go:452-469).
//
// Same decomposition as dx_gls.hip: k = k0 + k1 lambda2 (lambda2 = 6u^2, the
// eigenvalue of psi on G2 and of the Frobenius on GT), k0, k1 < 2^128.  Each
// half is recoded LSB-first into 17 signed digits in [-127, 128] (a byte plus
// the carry of the previous window), so one table per base holds
// d 2^(8w) Q for d = 1..128, w < 17 (2176 entries: 272 KiB on G2, 816 KiB on
// GT), and a negative digit uses the negated entry -- y -> -y on G2,
// conjugation (= inversion of a unitary element) on GT.  An evaluation costs
// 34 mixed additions / Fp12 products instead of the 44 of the 6-bit unsigned
// layout.  For the reference's random per-CN, per-column keys (99,360 points
// for a SPECTF-shaped query) the tables take ~111 GB of the 288 GB of HBM.
//
// Every body is force-inlined into an explicit __global__ kernel (no device
// calls: see dx_rpmsm.hip on branch relaxation in out-of-line callees).
#define DX_NI __host__ __device__ __forceinline__
#include "common.h"
#include "../bn254/gt_coop.h"

using namespace dxk;

namespace {
constexpr int kBits = 8;
constexpr int kHalf = 1 << (kBits - 1);   // 128 entries per window
constexpr int kWin = 17;                  // 16 bytes + the final carry
constexpr int kEnt = kWin * kHalf;        // 2176
constexpr int kWG = 64;

// k (8 limbs) = k0 + k1 * lambda2, k0 < lambda2 (4 limbs), k1 < 2^128: binary
// long division by the 127-bit constant.
DX_HD void split_lambda2(const uint32_t *k, uint32_t *k0, uint32_t *k1) {
  uint32_t rem[5] = {0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int bit = 255; bit >= 0; bit--) {
#pragma unroll
    for (int i = 4; i > 0; i--) rem[i] = (rem[i] << 1) | (rem[i - 1] >> 31);
    rem[0] = (rem[0] << 1) | ((k[bit >> 5] >> (bit & 31)) & 1u);
    uint32_t d[5], br = 0;
#pragma unroll
    for (int i = 0; i < 5; i++) d[i] = subb32(rem[i], i < 4 ? SIX_U2[i] : 0u, br);
    if (!br) {
#pragma unroll
      for (int i = 0; i < 5; i++) rem[i] = d[i];
      q[bit >> 5] |= 1u << (bit & 31);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; i++) k0[i] = rem[i];
  k0[4] = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) k1[i] = q[i];
}

// signed digit of byte window w (LSB first), carry in / out
DX_HD int sdigit(const uint32_t *k5, int w, uint32_t &carry) {
  const int bit = w * kBits;
  const uint32_t v = ((k5[bit >> 5] >> (bit & 31)) & 0xFFu) + carry;
  carry = v > (uint32_t)kHalf ? 1u : 0u;
  return carry ? (int)v - 256 : (int)v;
}

DX_HD G2J psi_j(const G2J &q) {
  return {mul(conj(q.x), Fp2::from_limbs(Frob::TWX1)), mul(conj(q.y), Fp2::from_limbs(Frob::TWY1)), conj(q.z)};
}

DX_HD void g2_half(G2J &a, const G2A *T, const uint32_t *k5) {
  uint32_t c = 0;
  for (int w = 0; w < kWin; w++) {
    const int d = sdigit(k5, w, c);
    if (d) {
      G2A q = T[w * kHalf + (d > 0 ? d : -d) - 1];
      if (d < 0) q.y = neg(q.y);
      a = jadd_mixed(a, q);
    }
  }
}

DX_HD G2J g2_gls8_eval(const G2A *T, const uint32_t *k) {
  uint32_t k0[5], k1[5];
  split_lambda2(k, k0, k1);
  G2J a = G2J::inf();
  g2_half(a, T, k1);
  a = psi_j(a);
  g2_half(a, T, k0);
  return a;
}

DX_HD void gt_half(Fp12 &f, const Fp12 *T, const uint32_t *k5) {
  uint32_t c = 0;
  for (int w = 0; w < kWin; w++) {
    const int d = sdigit(k5, w, c);
    if (d) {
      const Fp12 &e = T[w * kHalf + (d > 0 ? d : -d) - 1];
      f = mul(f, d > 0 ? e : conj(e));
    }
  }
}

DX_HD Fp12 gt_gls8_eval(const Fp12 *T, const uint32_t *k) {
  uint32_t k0[5], k1[5];
  split_lambda2(k, k0, k1);
  Fp12 f = Fp12::one();
  gt_half(f, T, k1);
  f = frob<1>(f);
  gt_half(f, T, k0);
  return f;
}

// ---- table construction: work[b*17 + w] = 2^(8w) base; entry = d * work
DX_HD void g2_pow_one(const uint32_t *bases_aff, uint32_t *work, int64_t b) {
  G2J acc = G2J::from_aff(at<G2A>(bases_aff, b));
  for (int w = 0; w < kWin; w++) {
    at<G2J>(work, b * kWin + w) = acc;
    for (int i = 0; i < kBits; i++) acc = jdbl(acc);
  }
}
DX_HD void gt_pow_one(const uint32_t *bases, uint32_t *work, int64_t b) {
  Fp12 acc = at<Fp12>(bases, b);
  for (int w = 0; w < kWin; w++) {
    at<Fp12>(work, b * kWin + w) = acc;
    for (int i = 0; i < kBits; i++) acc = cyclotomic_sqr(acc);
  }
}
// Entries by chunks of kCh consecutive digits d0 .. d0 + kCh - 1 of one
// window: the first by double-and-add from the window's base, each next one
// by one more addition / product -- ~1/7 of the per-entry double-and-add
// (setup: ~3.4 s of table building for a 3-CN SPECTF-shaped set).
constexpr int kCh = 16;
constexpr int kChunks = kEnt / kCh;  // 136 per base (kHalf = 128 is a multiple of kCh)

DX_HD void g2_entry_chunk_one(const uint32_t *work, uint32_t *table, int64_t t) {
  const int64_t b = t / kChunks, c = t % kChunks;
  const int w = (int)(c / (kHalf / kCh)), d0 = (int)(c % (kHalf / kCh)) * kCh + 1;
  const int64_t qi = b * kWin + w;  // q re-read per addition: no register copy to spill
  G2J acc = G2J::inf();
  for (int bit = kBits - 1; bit >= 0; bit--) {
    acc = jdbl(acc);
    if ((d0 >> bit) & 1) acc = jadd(acc, at<G2J>(work, qi));
  }
  const int64_t e0 = b * kEnt + (int64_t)w * kHalf + d0 - 1;
  for (int j = 0; j < kCh; j++) {
    at<G2A>(table, e0 + j) = to_affine(acc);
    if (j + 1 < kCh) acc = jadd(acc, at<G2J>(work, qi));
  }
}

DX_HD void gt_entry_chunk_one(const uint32_t *work, uint32_t *table, int64_t t) {
  const int64_t b = t / kChunks, c = t % kChunks;
  const int w = (int)(c / (kHalf / kCh)), d0 = (int)(c % (kHalf / kCh)) * kCh + 1;
  const Fp12 q = at<Fp12>(work, b * kWin + w);
  Fp12 acc = Fp12::one();
  for (int bit = kBits - 1; bit >= 0; bit--) {
    acc = cyclotomic_sqr(acc);
    if ((d0 >> bit) & 1) acc = mul(acc, q);
  }
  const int64_t e0 = b * kEnt + (int64_t)w * kHalf + d0 - 1;
  for (int j = 0; j < kCh; j++) {
    at<Fp12>(table, e0 + j) = acc;
    if (j + 1 < kCh) acc = mul(acc, q);
  }
}

// the GT chunks on three lanes per chunk (gt_coop.h: no Fp12 spills)
__global__ void __launch_bounds__(64) DX_OCC gt_entry_chunk_coop(const uint32_t *work, uint32_t *table, int64_t n) {
  const coop::Role R = coop::role();
  const int64_t t = (int64_t)blockIdx.x * coop::kTriples + R.g;
  if (R.g >= coop::kTriples || t >= n) return;  // whole triples leave together
  const int64_t b = t / kChunks, c = t % kChunks;
  const int w = (int)(c / (kHalf / kCh)), d0 = (int)(c % (kHalf / kCh)) * kCh + 1;
  const Fp12 *Q = &at<Fp12>(work, b * kWin + w);  // re-read per product (L1 / L2): no register copy to spill
  Fp6 acc = coop::one(R);
  for (int bit = kBits - 1; bit >= 0; bit--) {
    coop::mul(acc, acc, R);
    if ((d0 >> bit) & 1) coop::mul(acc, coop::load(Q, false, R), R);
  }
  const int64_t e0 = b * kEnt + (int64_t)w * kHalf + d0 - 1;
  for (int j = 0; j < kCh; j++) {
    coop::store(&at<Fp12>(table, e0 + j), acc, R);
    if (j + 1 < kCh) coop::mul(acc, coop::load(Q, false, R), R);
  }
}

DX_HD void g2_mul_one(const uint32_t *tables, const int32_t *tab_idx, const uint32_t *scalars, uint32_t *out_aff,
                      int64_t i) {
  const G2A *T = reinterpret_cast<const G2A *>(tables) + (int64_t)(tab_idx ? tab_idx[i] : 0) * kEnt;
  at<G2A>(out_aff, i) = to_affine(g2_gls8_eval(T, scalars + 8 * i));
}

// ---- gT with signed 16-bit windows: T16[w*32768 + d-1] = gT^(d 2^(16w)),
// d = 1..32768, w < 17 (214 MB, one table per device): 17 products per
// exponentiation instead of the 32 of the 8-bit comb
constexpr int kB16 = 16, kH16 = 1 << 15, kW16 = 17;
DX_HD void gt16_entry_one(const uint32_t *pow2, uint32_t *table, int64_t t) {
  const int w = (int)(t / kH16), d = (int)(t % kH16) + 1;
  const Fp12 q = at<Fp12>(pow2, w);
  Fp12 acc = Fp12::one();
  for (int bit = kB16 - 1; bit >= 0; bit--) {  // d <= 2^15
    acc = cyclotomic_sqr(acc);
    if ((d >> bit) & 1) acc = mul(acc, q);
  }
  at<Fp12>(table, t) = acc;
}
DX_HD Fp12 gt16_pow(const Fp12 *T, const uint32_t *k) {
  Fp12 f = Fp12::one();
  uint32_t carry = 0;
  for (int w = 0; w < kW16; w++) {
    const uint32_t raw = w < 16 ? (k[w >> 1] >> (16 * (w & 1))) & 0xFFFFu : 0u;
    const uint32_t v = raw + carry;
    carry = v > (uint32_t)kH16 ? 1u : 0u;
    const int d = carry ? (int)v - 65536 : (int)v;
    if (d) {
      const Fp12 &e = T[w * kH16 + (d > 0 ? d : -d) - 1];
      f = mul(f, d > 0 ? e : conj(e));
    }
  }
  return f;
}

// prover pass 1: a[p*S*L + j] = gT^(t[p*L + j]) (shared by the S servers);
// t16: gt_table is the signed 16-bit table instead of the 8-bit comb
DX_HD void prove_t_one(const uint32_t *t_sc, const uint32_t *gt_table, uint32_t *a_out, int S, int L, int t16,
                       int64_t pj) {
  const int64_t p = pj / L, j = pj % L;
  const Fp12 *T = reinterpret_cast<const Fp12 *>(gt_table);
  at<Fp12>(a_out, p * S * L + j) = t16 ? gt16_pow(T, t_sc + 8 * pj) : gt_fixed_pow(T, t_sc + 8 * pj);
}
// prover pass 2 over the items of one server range [i_lo, i_hi): a[it] = E^(e[it]) * a[p*S*L + j]
DX_HD void prove_e_one(const uint32_t *gphi_tables, const int32_t *tab_idx, const uint32_t *e_sc, uint32_t *a_out,
                       int S, int L, int i_lo, int i_hi, int64_t k) {
  const int64_t per = (int64_t)(i_hi - i_lo) * L;
  const int64_t p = k / per, r = k % per;
  const int64_t i = i_lo + r / L, j = r % L;
  const int64_t it = (p * S + i) * L + j;
  const Fp12 *T = reinterpret_cast<const Fp12 *>(gphi_tables) + (int64_t)tab_idx[it] * kEnt;
  at<Fp12>(a_out, it) = mul(gt_gls8_eval(T, e_sc + 8 * it), at<Fp12>(a_out, p * S * L + j));
}

// ---- the two prover passes on the GPU: three lanes per item (gt_coop.h)
// x <- x * prod of the signed 8-bit windows of one 128-bit half (role operands)
__device__ __forceinline__ void gt_half_coop(Fp6 &x, const Fp12 *T, const uint32_t *k5, const coop::Role &R) {
  uint32_t c = 0;
  for (int w = 0; w < kWin; w++) {
    const int d = sdigit(k5, w, c);
    if (d) coop::mul(x, coop::load(&T[w * kHalf + (d > 0 ? d : -d) - 1], d < 0, R), R);
  }
}

__global__ void __launch_bounds__(kWG) DX_OCC prove_t_coop(const uint32_t *t_sc, const uint32_t *gt16, uint32_t *a_out,
                                                          int S, int L, int64_t n_pj) {
  const coop::Role R = coop::role();
  const int64_t pj = (int64_t)blockIdx.x * coop::kTriples + R.g;
  if (R.g >= coop::kTriples || pj >= n_pj) return;  // whole triples leave together
  const Fp12 *T = reinterpret_cast<const Fp12 *>(gt16);
  const uint32_t *k = t_sc + 8 * pj;
  Fp6 x = coop::one(R);
  uint32_t carry = 0;
  for (int w = 0; w < kW16; w++) {
    const uint32_t raw = w < 16 ? (k[w >> 1] >> (16 * (w & 1))) & 0xFFFFu : 0u;
    const uint32_t v = raw + carry;
    carry = v > (uint32_t)kH16 ? 1u : 0u;
    const int d = carry ? (int)v - 65536 : (int)v;
    if (d) coop::mul(x, coop::load(&T[w * kH16 + (d > 0 ? d : -d) - 1], d < 0, R), R);
  }
  const int64_t p = pj / L, j = pj % L;
  coop::store(&at<Fp12>(a_out, p * S * L + j), x, R);
}

// server range [i_lo, i_hi): a[it] = E_phi(it)^(e[it]) * a[p*S*L + j]
__global__ void __launch_bounds__(kWG) DX_OCC prove_e_coop(const uint32_t *gphi, const int32_t *tab_idx,
                                                          const uint32_t *e_sc, uint32_t *a_out, int S, int L,
                                                          int i_lo, int i_hi, int64_t n) {
  const coop::Role R = coop::role();
  const int64_t kk = (int64_t)blockIdx.x * coop::kTriples + R.g;
  if (R.g >= coop::kTriples || kk >= n) return;
  const int64_t per = (int64_t)(i_hi - i_lo) * L;
  const int64_t p = kk / per, rr = kk % per;
  const int64_t i = i_lo + rr / L, j = rr % L;
  const int64_t it = (p * S + i) * L + j;
  const Fp12 *T = reinterpret_cast<const Fp12 *>(gphi) + (int64_t)tab_idx[it] * kEnt;
  uint32_t k0[5], k1[5];
  split_lambda2(e_sc + 8 * it, k0, k1);
  Fp6 x = coop::one(R);
  gt_half_coop(x, T, k1, R);
  coop::frob1(x, R);
  gt_half_coop(x, T, k0, R);
  Fp12 *slot = &at<Fp12>(a_out, p * S * L + j);
  coop::mul(x, coop::load(slot, false, R), R);  // every role has read the shared slot before any store
  coop::store(&at<Fp12>(a_out, it), x, R);
}

#define DX_TID() const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x
__global__ void __launch_bounds__(kWG) DX_OCC g2_pow_kernel(const uint32_t *b, uint32_t *w, int64_t n) {
  DX_TID();
  if (i < n) g2_pow_one(b, w, i);
}
__global__ void __launch_bounds__(kWG) DX_OCC g2_entry_chunk_kernel(const uint32_t *w, uint32_t *t, int64_t n) {
  DX_TID();
  if (i < n) g2_entry_chunk_one(w, t, i);
}
__global__ void __launch_bounds__(kWG) DX_OCC gt_pow_kernel(const uint32_t *b, uint32_t *w, int64_t n) {
  DX_TID();
  if (i < n) gt_pow_one(b, w, i);
}

__global__ void __launch_bounds__(kWG) DX_OCC g2_mul_kernel(const uint32_t *tables, const int32_t *tab_idx,
                                                           const uint32_t *sc, uint32_t *out, int64_t n) {
  DX_TID();
  if (i < n) g2_mul_one(tables, tab_idx, sc, out, i);
}
// chunks of kCh consecutive digits per lane triple (as gt_entry_chunk_coop)
__global__ void __launch_bounds__(64) DX_OCC gt16_entry_chunk_coop(const uint32_t *pow2, uint32_t *table, int64_t n) {
  const coop::Role R = coop::role();
  const int64_t t = (int64_t)blockIdx.x * coop::kTriples + R.g;
  if (R.g >= coop::kTriples || t >= n) return;
  const int w = (int)(t / (kH16 / kCh)), d0 = (int)(t % (kH16 / kCh)) * kCh + 1;
  const Fp12 *Q = &at<Fp12>(pow2, w);
  Fp6 acc = coop::one(R);
  for (int bit = kB16 - 1; bit >= 0; bit--) {
    coop::mul(acc, acc, R);
    if ((d0 >> bit) & 1) coop::mul(acc, coop::load(Q, false, R), R);
  }
  const int64_t e0 = (int64_t)w * kH16 + d0 - 1;
  for (int j = 0; j < kCh; j++) {
    coop::store(&at<Fp12>(table, e0 + j), acc, R);
    if (j + 1 < kCh) coop::mul(acc, coop::load(Q, false, R), R);
  }
}
#undef DX_TID

inline dim3 grid_of(int64_t n) { return dim3((unsigned)((n + kWG - 1) / kWG)); }
inline dim3 grid_coop(int64_t n) { return dim3((unsigned)((n + coop::kTriples - 1) / coop::kTriples)); }

}  // namespace

extern "C" {
int dx_gls8_entries() { return kEnt; }
int dx_gt16_entries() { return kW16 * kH16; }

// pow2[w] = gT^(2^(16w)) for w < 17 (host-computed), table [17*32768, 96]
int dx_gt16_table(int on_gpu, void *stream, const uint32_t *pow2, uint32_t *table) {
  const int64_t n = (int64_t)kW16 * kH16;
  if (!on_gpu) {
    host_for_each(n, [=](int64_t t) { gt16_entry_one(pow2, table, t); });
    return 0;
  }
  hipLaunchKernelGGL(gt16_entry_chunk_coop, grid_coop(n / kCh), dim3(kWG), 0, (hipStream_t)stream, pow2, table,
                     n / kCh);
  return check_hip(hipGetLastError(), "gt16_table");
}

// table[b*2176 + w*128 + d-1] = d 2^(8w) A_b (affine); work [nb*17] Jacobian
int dx_g2_gls8_table(int on_gpu, void *stream, const uint32_t *bases_aff, uint32_t *work, uint32_t *table,
                     int64_t n_bases) {
  if (n_bases <= 0) return 0;
  if (!on_gpu) {
    host_for_each(n_bases, [=](int64_t b) { g2_pow_one(bases_aff, work, b); });
    host_for_each(n_bases * kChunks, [=](int64_t t) { g2_entry_chunk_one(work, table, t); });
    return 0;
  }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(g2_pow_kernel, grid_of(n_bases), dim3(kWG), 0, s, bases_aff, work, n_bases);
  hipLaunchKernelGGL(g2_entry_chunk_kernel, grid_of(n_bases * kChunks), dim3(kWG), 0, s, work, table,
                     n_bases * kChunks);
  return check_hip(hipGetLastError(), "g2_gls8_table");
}

// table[b*2176 + w*128 + d-1] = E_b^(d 2^(8w)); work [nb*17]
int dx_gt_gls8_table(int on_gpu, void *stream, const uint32_t *bases, uint32_t *work, uint32_t *table,
                     int64_t n_bases) {
  if (n_bases <= 0) return 0;
  if (!on_gpu) {
    host_for_each(n_bases, [=](int64_t b) { gt_pow_one(bases, work, b); });
    host_for_each(n_bases * kChunks, [=](int64_t t) { gt_entry_chunk_one(work, table, t); });
    return 0;
  }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(gt_pow_kernel, grid_of(n_bases), dim3(kWG), 0, s, bases, work, n_bases);
  hipLaunchKernelGGL(gt_entry_chunk_coop, grid_coop(n_bases * kChunks), dim3(kWG), 0, s, work, table,
                     n_bases * kChunks);
  return check_hip(hipGetLastError(), "gt_gls8_table");
}

int dx_g2_gls8_mul(int on_gpu, void *stream, const uint32_t *tables, const int32_t *tab_idx, const uint32_t *scalars,
                   uint32_t *out_aff, int64_t n) {
  if (n <= 0) return 0;
  if (!on_gpu) {
    host_for_each(n, [=](int64_t i) { g2_mul_one(tables, tab_idx, scalars, out_aff, i); });
    return 0;
  }
  hipLaunchKernelGGL(g2_mul_kernel, grid_of(n), dim3(kWG), 0, (hipStream_t)stream, tables, tab_idx, scalars, out_aff,
                     n);
  return check_hip(hipGetLastError(), "g2_gls8_mul");
}

// a[it] = E_phi(it)^(e[it]) * gT^(t[p, j]): the gT^t part once per (p, j), then
// the servers i >= 1 and server 0 in two launches (server 0's slot holds gT^t
// until its own launch overwrites it last).
int dx_rp_prove_a_gls8(int on_gpu, void *stream, const uint32_t *gphi_tables, const int32_t *tab_idx,
                       const uint32_t *e_sc, const uint32_t *t_sc, const uint32_t *gt_table, uint32_t *a_out,
                       int64_t n_items, int S, int L, int t16) {
  if (n_items <= 0) return 0;
  const int64_t n_pj = n_items / S, n_p = n_pj / L;
  const int ranges[2][2] = {{1, S}, {0, 1}};
  if (!on_gpu) {
    host_for_each(n_pj, [=](int64_t pj) { prove_t_one(t_sc, gt_table, a_out, S, L, t16, pj); });
    for (auto &rg : ranges) {
      const int lo = rg[0], hi = rg[1];
      if (hi <= lo) continue;
      host_for_each(n_p * (hi - lo) * L,
                    [=](int64_t k) { prove_e_one(gphi_tables, tab_idx, e_sc, a_out, S, L, lo, hi, k); });
    }
    return 0;
  }
  hipStream_t s = (hipStream_t)stream;
  if (!t16) return check_hip(hipErrorInvalidValue, "rp_prove_a_gls8 (the GPU path takes the 16-bit gT table)");
  hipLaunchKernelGGL(prove_t_coop, grid_coop(n_pj), dim3(kWG), 0, s, t_sc, gt_table, a_out, S, L, n_pj);
  for (auto &rg : ranges) {
    const int lo = rg[0], hi = rg[1];
    if (hi <= lo) continue;
    const int64_t n = n_p * (hi - lo) * L;
    hipLaunchKernelGGL(prove_e_coop, grid_coop(n), dim3(kWG), 0, s, gphi_tables, tab_idx, e_sc, a_out, S, L, lo, hi,
                       n);
  }
  return check_hip(hipGetLastError(), "rp_prove_a_gls8");
}
}  // extern "C"
