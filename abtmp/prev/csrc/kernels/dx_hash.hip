// Device CSPRNG (K17) and chunked SHA-256 payload digests (K12).
//
// dx_random_scalars: uniform Fr scalars from ChaCha20 (RFC 8439 block function,
//   key = 256 fresh bits from the OS CSPRNG per call, nonce = 0, counter =
//   item index).  Each item consumes one 64-byte block read as a 512-bit
//   integer x = lo + 2^256 hi and returns x mod r = lo + hi * (2^256 mod r)
//   (statistical distance from uniform ~ 2^-258, no rejection loop, so every
//   thread does the same work).  Reference: every
//   ``Scalar().Pick(suite.RandomStream())`` of the Go code (16 sites) --
//   kyber reads from crypto/rand; here one launch fills a whole proof batch.
//
// dx_sha256_chunks: SHA-256 of every `chunk`-byte slice of a payload, one
//   thread per slice (the last slice may be short).  The proof-envelope digest
//   that a DP/CN Schnorr-signs and a VN re-checks (structs_proofs.go:117-143,
//   :498-505 sign/verify the marshalled proof) is defined as
//   SHA-256("DXTH1" || le64(len) || le64(chunk) || H(slice_0) || H(slice_1) ...);
//   for a range-proof bundle (tens of MB of pairing-group elements) the slices
//   are hashed where the bytes already live -- in HBM -- and only the slice
//   digests (32 B per 4 KiB) cross to the host.
#include "common.h"

using namespace dxk;

namespace {

DX_HD uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
DX_HD uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

#define DX_QR(a, b, c, d)          \
  a += b; d ^= a; d = rotl32(d, 16); \
  c += d; b ^= c; b = rotl32(b, 12); \
  a += b; d ^= a; d = rotl32(d, 8);  \
  c += d; b ^= c; b = rotl32(b, 7);

DX_HD void chacha20_block(const uint32_t key[8], uint32_t counter, uint32_t out[16]) {
  uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                    key[4],      key[5],      key[6],      key[7],      counter, 0u,     0u,     0u};
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = s[i];
#pragma unroll
  for (int r = 0; r < 10; r++) {
    DX_QR(x[0], x[4], x[8], x[12]);
    DX_QR(x[1], x[5], x[9], x[13]);
    DX_QR(x[2], x[6], x[10], x[14]);
    DX_QR(x[3], x[7], x[11], x[15]);
    DX_QR(x[0], x[5], x[10], x[15]);
    DX_QR(x[1], x[6], x[11], x[12]);
    DX_QR(x[2], x[7], x[8], x[13]);
    DX_QR(x[3], x[4], x[9], x[14]);
  }
#pragma unroll
  for (int i = 0; i < 16; i++) out[i] = x[i] + s[i];
}
#undef DX_QR

// ---------------------------------------------------------------- SHA-256
struct Sha256 {
  uint32_t h[8];
  DX_HD void init() {
    h[0] = 0x6a09e667u; h[1] = 0xbb67ae85u; h[2] = 0x3c6ef372u; h[3] = 0xa54ff53au;
    h[4] = 0x510e527fu; h[5] = 0x9b05688cu; h[6] = 0x1f83d9abu; h[7] = 0x5be0cd19u;
  }
  // w: 16 big-endian message words
  DX_HD void compress(uint32_t w[16]) {
    // round constants as an unrolled immediate sequence (no memory table, so the
    // same function serves the host path and the gfx950 kernels)
    constexpr uint32_t K[64] = {
        0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
        0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
        0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
        0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
        0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
        0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
        0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
        0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
    for (int i = 0; i < 64; i++) {
      uint32_t wi;
      if (i < 16) {
        wi = w[i];
      } else {
        uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
        uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
        uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
        wi = w[i & 15] = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      }
      uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
      uint32_t ch = (e & f) ^ (~e & g);
      uint32_t t1 = hh + S1 + ch + K[i] + wi;
      uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
      uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
      uint32_t t2 = S0 + mj;
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
};

DX_HD uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

// SHA-256 of p[0..len), p 4-byte aligned; digest as 8 big-endian words.
DX_HD void sha256_bytes(const uint8_t *p, int64_t len, uint32_t out[8]) {
  Sha256 st;
  st.init();
  uint32_t w[16];
  int64_t full = len / 64;
  const uint32_t *p32 = reinterpret_cast<const uint32_t *>(p);
  for (int64_t blk = 0; blk < full; blk++) {
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = bswap32(p32[blk * 16 + i]);
    st.compress(w);
  }
  // tail + padding (1 or 2 blocks)
  const int64_t rem = len - full * 64;
  const uint8_t *t = p + full * 64;
  uint8_t buf[128];
  for (int i = 0; i < 128; i++) buf[i] = 0;
  for (int64_t i = 0; i < rem; i++) buf[i] = t[i];
  buf[rem] = 0x80;
  const int nblk = rem + 9 <= 64 ? 1 : 2;
  const uint64_t bits = (uint64_t)len * 8ull;
  for (int i = 0; i < 8; i++) buf[nblk * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
  for (int b = 0; b < nblk; b++) {
    for (int i = 0; i < 16; i++)
      w[i] = ((uint32_t)buf[b * 64 + 4 * i] << 24) | ((uint32_t)buf[b * 64 + 4 * i + 1] << 16) |
             ((uint32_t)buf[b * 64 + 4 * i + 2] << 8) | (uint32_t)buf[b * 64 + 4 * i + 3];
    st.compress(w);
  }
  for (int i = 0; i < 8; i++) out[i] = st.h[i];
}

// Tail (last partial block + padding) of a slice whose full blocks are
// already compressed into st.
DX_HD void sha256_tail(Sha256 &st, const uint8_t *p, int64_t len, uint32_t out[8]) {
  const int64_t full = len / 64;
  const int64_t rem = len - full * 64;
  const uint8_t *t = p + full * 64;
  uint8_t buf[128];
  for (int i = 0; i < 128; i++) buf[i] = 0;
  for (int64_t i = 0; i < rem; i++) buf[i] = t[i];
  buf[rem] = 0x80;
  const int nblk = rem + 9 <= 64 ? 1 : 2;
  const uint64_t bits = (uint64_t)len * 8ull;
  for (int i = 0; i < 8; i++) buf[nblk * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
  uint32_t w[16];
  for (int b = 0; b < nblk; b++) {
    for (int i = 0; i < 16; i++)
      w[i] = ((uint32_t)buf[b * 64 + 4 * i] << 24) | ((uint32_t)buf[b * 64 + 4 * i + 1] << 16) |
             ((uint32_t)buf[b * 64 + 4 * i + 2] << 8) | (uint32_t)buf[b * 64 + 4 * i + 3];
    st.compress(w);
  }
  for (int i = 0; i < 8; i++) out[i] = st.h[i];
}

// Slice hashing on the GPU with coalesced loads: one slice per lane (4 KiB
// apart), but each 64-byte message block of the 64 lanes' slices is first
// staged in LDS by 16-lane groups reading one slice's block contiguously (4
// slices per load instruction) -- a lane reading its own slice directly makes
// every load touch 64 cache lines (~80 GB/s for a VN's 470 MB of slice
// digests).  ``desc(t, p, m)`` names slice t's bytes; the partial last block
// and the padding are hashed per lane from global memory.
template <class Desc>
__global__ void __launch_bounds__(64) sha_slices_kernel(Desc desc, int64_t total, uint32_t *out) {
  __shared__ uint32_t tile[64][17];
  __shared__ const uint8_t *sp[64];
  __shared__ int64_t snf[64];
  const int lane = threadIdx.x;
  const int64_t t = (int64_t)blockIdx.x * 64 + lane;
  const uint8_t *p = nullptr;
  int64_t m = 0;
  if (t < total) desc(t, p, m);
  if (m < 0) m = 0;
  const int64_t nfull = m / 64;
  sp[lane] = p;
  snf[lane] = nfull;
  __syncthreads();
  int64_t maxfull = 0;
  for (int i = 0; i < 64; i++) maxfull = snf[i] > maxfull ? snf[i] : maxfull;
  Sha256 st;
  st.init();
  const int q = lane & 15;
  for (int64_t b = 0; b < maxfull; b++) {
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int src = r * 4 + (lane >> 4);
      if (b < snf[src]) tile[src][q] = reinterpret_cast<const uint32_t *>(sp[src] + b * 64)[q];
    }
    __syncthreads();
    if (b < nfull) {
      uint32_t w[16];
#pragma unroll
      for (int i = 0; i < 16; i++) w[i] = bswap32(tile[lane][i]);
      st.compress(w);
    }
    __syncthreads();
  }
  if (t < total) {
    uint32_t d[8];
    sha256_tail(st, p, m, d);
    for (int k = 0; k < 8; k++) out[8 * t + k] = d[k];
  }
}

template <class Desc>
int sha_slices(void *stream, const Desc &desc, int64_t total, uint32_t *out, const char *name) {
  if (total <= 0) return 0;
  hipLaunchKernelGGL(sha_slices_kernel<Desc>, dim3((unsigned)((total + 63) / 64)), dim3(64), 0, (hipStream_t)stream,
                     desc, total, out);
  return check_hip(hipGetLastError(), name);
}

}  // namespace

extern "C" int dx_random_scalars(int on_gpu, void *stream, const uint32_t *key_host, uint32_t counter0, uint32_t *out,
                                 int64_t n) {
  struct K8 {
    uint32_t k[8];
  } kk;
  for (int i = 0; i < 8; i++) kk.k[i] = key_host[i];
  auto op = [=] __host__ __device__(int64_t i) {
    uint32_t blk[16];
    chacha20_block(kk.k, counter0 + (uint32_t)i, blk);
    Fr lo = reduce_256<FrParams>(blk);
    Fr hi = reduce_256<FrParams>(blk + 8);
    // hi * 2^256 mod r == to_mont(hi); plain-form result
    Fr x = fadd(lo, to_mont(hi));
    if (x.is_zero()) x.v[0] = 1;  // never 0 (probability 2^-254)
    at<Fr>(out, i) = x;
  };
  return run(on_gpu, stream, n, op, false, "random_scalars");
}

// GLV batch weights straight from the generator (one launch instead of the
// generator + slicing + two Fr ops): item i's scalar x_i exactly as
// dx_random_scalars draws it, a = limb 0 and b = limb 1 of x_i (32-bit
// halves), rho_i = a + b * lambda mod r.  lam: lambda as 8 canonical limbs.
extern "C" int dx_prg_glv(int on_gpu, void *stream, const uint32_t *key_host, uint32_t counter0, const uint32_t *lam_host,
                          int32_t *ab, uint32_t *rho, int64_t n) {
  struct K8 {
    uint32_t k[8];
  } kk, ll;
  for (int i = 0; i < 8; i++) {
    kk.k[i] = key_host[i];
    ll.k[i] = lam_host[i];
  }
  auto op = [=] __host__ __device__(int64_t i) {
    uint32_t blk[16];
    chacha20_block(kk.k, counter0 + (uint32_t)i, blk);
    Fr lo = reduce_256<FrParams>(blk);
    Fr hi = reduce_256<FrParams>(blk + 8);
    Fr x = fadd(lo, to_mont(hi));
    if (x.is_zero()) x.v[0] = 1;
    const uint32_t a = x.v[0], b = x.v[1];
    ab[2 * i] = (int32_t)a;
    ab[2 * i + 1] = (int32_t)b;
    uint32_t wa[8] = {a, 0, 0, 0, 0, 0, 0, 0}, wb[8] = {b, 0, 0, 0, 0, 0, 0, 0};
    const Fr A = reduce_256<FrParams>(wa), B = reduce_256<FrParams>(wb), L = reduce_256<FrParams>(ll.k);
    at<Fr>(rho, i) = fadd(A, fmul(B, to_mont(L)));
  };
  return run(on_gpu, stream, n, op, false, "prg_glv");
}

// Low-``bits`` batch weights straight from the generator: item i's scalar as
// dx_random_scalars draws it, with every bit from ``bits`` up cleared (the
// GT-membership combinations, 64-bit D weights) -- one launch instead of the
// generator plus masking kernels.
extern "C" int dx_prg_bits(int on_gpu, void *stream, const uint32_t *key_host, uint32_t counter0, int bits,
                           uint32_t *out, int64_t n) {
  if (bits < 0 || bits > 256) return -2;
  struct K8 {
    uint32_t k[8];
  } kk;
  for (int i = 0; i < 8; i++) kk.k[i] = key_host[i];
  auto op = [=] __host__ __device__(int64_t i) {
    uint32_t blk[16];
    chacha20_block(kk.k, counter0 + (uint32_t)i, blk);
    Fr lo = reduce_256<FrParams>(blk);
    Fr hi = reduce_256<FrParams>(blk + 8);
    Fr x = fadd(lo, to_mont(hi));
    if (x.is_zero()) x.v[0] = 1;
    for (int w = 0; w < 8; w++) {
      const int lo_bit = 32 * w;
      uint32_t v = x.v[w];
      if (lo_bit >= bits) v = 0;
      else if (bits - lo_bit < 32) v &= (1u << (bits - lo_bit)) - 1u;
      out[8 * i + w] = v;
    }
  };
  return run(on_gpu, stream, n, op, false, "prg_bits");
}

// out[i] = 8 big-endian words of SHA-256(data[i*chunk, min(len, (i+1)*chunk)))
extern "C" int dx_sha256_chunks(int on_gpu, void *stream, const uint8_t *data, int64_t len, int64_t chunk,
                                uint32_t *out) {
  if (chunk <= 0 || (chunk & 63) != 0) return -2;
  const int64_t n = len == 0 ? 1 : (len + chunk - 1) / chunk;
  auto op = [=] __host__ __device__(int64_t i) {
    const int64_t off = i * chunk;
    const int64_t m = len - off < chunk ? len - off : chunk;
    uint32_t d[8];
    sha256_bytes(data + off, m, d);
    for (int k = 0; k < 8; k++) out[8 * i + k] = d[k];
  };
  if (on_gpu) {
    auto desc = [=] __device__(int64_t i, const uint8_t *&p, int64_t &m) {
      const int64_t off = i * chunk;
      p = data + off;
      m = len - off < chunk ? len - off : chunk;
    };
    return sha_slices(stream, desc, n, out, "sha256_chunks");
  }
  return run(on_gpu, stream, n, op, false, "sha256_chunks");
}

// The same slice digests for `rows` equally long payloads laid out every
// `stride` bytes (one envelope per DP of a batch): out[(r*k + i)*8 ..] with
// k = ceil(len / chunk) slices per row (1 for an empty payload).
extern "C" int dx_sha256_rows(int on_gpu, void *stream, const uint8_t *data, int64_t rows, int64_t stride,
                              int64_t len, int64_t chunk, uint32_t *out) {
  if (chunk <= 0 || (chunk & 63) != 0 || rows < 0 || stride < len) return -2;
  const int64_t k = len == 0 ? 1 : (len + chunk - 1) / chunk;
  auto op = [=] __host__ __device__(int64_t t) {
    const int64_t r = t / k, i = t - r * k;
    const int64_t off = i * chunk;
    const int64_t m = len - off < chunk ? len - off : chunk;
    uint32_t d[8];
    sha256_bytes(data + r * stride + off, m, d);
    for (int q = 0; q < 8; q++) out[8 * t + q] = d[q];
  };
  if (on_gpu) {
    auto desc = [=] __device__(int64_t t, const uint8_t *&p, int64_t &m) {
      const int64_t r = t / k, i = t - r * k;
      const int64_t off = i * chunk;
      p = data + r * stride + off;
      m = len - off < chunk ? len - off : chunk;
    };
    return sha_slices(stream, desc, rows * k, out, "sha256_rows");
  }
  return run(on_gpu, stream, rows * k, op, false, "sha256_rows");
}

// Slice digests of MANY payloads in one launch (a VN inbox: every proof
// envelope of every CN / DP, and the transcripts inside them).  seg[3*q ..]
// = (address, byte length, first output slice) of payload q, in ascending
// first-slice order; every payload has ceil(len / chunk) slices (1 if empty).
// One thread per slice finds its payload by binary search.
extern "C" int dx_sha256_segments(int on_gpu, void *stream, const int64_t *seg, int64_t n_seg, int64_t total,
                                  int64_t chunk, uint32_t *out) {
  if (chunk <= 0 || (chunk & 63) != 0 || n_seg <= 0) return -2;
  auto op = [=] __host__ __device__(int64_t t) {
    int64_t lo = 0, hi = n_seg - 1;
    while (lo < hi) {  // last segment whose first slice <= t
      const int64_t mid = (lo + hi + 1) >> 1;
      if (seg[3 * mid + 2] <= t) lo = mid;
      else hi = mid - 1;
    }
    const uint8_t *base = (const uint8_t *)(uintptr_t)seg[3 * lo];
    const int64_t len = seg[3 * lo + 1];
    const int64_t off = (t - seg[3 * lo + 2]) * chunk;
    const int64_t m = len - off < chunk ? len - off : chunk;
    uint32_t d[8];
    sha256_bytes(base + off, m > 0 ? m : 0, d);
    for (int q = 0; q < 8; q++) out[8 * t + q] = d[q];
  };
  if (on_gpu) {
    auto desc = [=] __device__(int64_t t, const uint8_t *&p, int64_t &m) {
      int64_t lo = 0, hi = n_seg - 1;
      while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (seg[3 * mid + 2] <= t) lo = mid;
        else hi = mid - 1;
      }
      const int64_t len = seg[3 * lo + 1];
      const int64_t off = (t - seg[3 * lo + 2]) * chunk;
      p = (const uint8_t *)(uintptr_t)seg[3 * lo] + off;
      m = len - off < chunk ? len - off : chunk;
    };
    return sha_slices(stream, desc, total, out, "sha256_segments");
  }
  return run(on_gpu, stream, total, op, false, "sha256_segments");
}

// Independent G1 generators h_i (unknown discrete logs) for commitment
// schemes -- the permutation commitments of the shuffle proof.  For index i:
// ctr = 0, 1, ...: x = SHA-256(seed || le64(i) || le32(ctr)) (big endian) mod p;
// accept when x^3 + 3 is a square, y = (x^3+3)^((p+1)/4) with even canonical y.
// BN254 G1 has cofactor 1, so every curve point is a generator.  Mirrored by
// drynx_amd/proofs/shuffle.py:_hash_to_g1_index (host oracle).
extern "C" int dx_hash_to_g1(int on_gpu, void *stream, const uint32_t *seed_host, const uint32_t *sqrt_exp_host,
                             int64_t start, uint32_t *out_aff, int64_t n) {
  struct Args {
    uint32_t seed[8], e[8];
  } A;
  for (int i = 0; i < 8; i++) {
    A.seed[i] = seed_host[i];
    A.e[i] = sqrt_exp_host[i];
  }
  auto op = [=] __host__ __device__(int64_t k) {
    const uint64_t idx = (uint64_t)(start + k);
    G1A res = G1A::inf();
    for (uint32_t ctr = 0; ctr < 128; ctr++) {
      // one 44-byte message in one padded block
      uint32_t w[16];
      for (int i = 0; i < 8; i++) w[i] = A.seed[i];  // seed bytes as big-endian message words
      w[8] = bswap32((uint32_t)idx);
      w[9] = bswap32((uint32_t)(idx >> 32));
      w[10] = bswap32(ctr);
      w[11] = 0x80000000u;
      for (int i = 12; i < 15; i++) w[i] = 0;
      w[15] = 44 * 8;
      Sha256 st;
      st.init();
      st.compress(w);
      uint32_t le[8];
      for (int i = 0; i < 8; i++) le[i] = st.h[7 - i];  // big-endian digest -> little-endian limbs
      Fp x = to_mont(reduce_256<FpParams>(le));
      Fp rhs = fadd(fmul(fsqr(x), x), Fp::from_limbs(Curve::B1));
      Fp y = fpow(rhs, A.e);
      if (fsqr(y) == rhs) {
        if (from_mont(y).v[0] & 1u) y = fneg(y);
        res = {x, y};
        break;
      }
    }
    at<G1A>(out_aff, k) = res;
  };
  return run(on_gpu, stream, n, op, true, "hash_to_g1");
}
