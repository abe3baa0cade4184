// Range-proof Fiat-Shamir challenges on the device: SHA3-512 (Keccak-f[1600],
// FIPS 202) of B || C || Y per value, reduced mod r.
//
// Reference: lib/range/range_proof.go:350-374 -- c = SetBytes(SHA3-512(
// B.MarshalBinary() || Commit.C.MarshalBinary() || (sum_i y_i).MarshalBinary()))
// mod r, one hash per encrypted value.  The prover computed these on the host
// (one hashlib call per value: ~3.4 ms for the 2070 values of an LR query, on
// the query's critical path); here one thread per value hashes the 192-byte
// message where the commitments already live.
#include "common.h"

namespace {

DX_HD uint64_t rotl64(uint64_t x, int n) { return n == 0 ? x : (x << n) | (x >> (64 - n)); }
DX_HD uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

DX_HD void keccak_f1600(uint64_t a[25]) {
  constexpr uint64_t RC[24] = {
      0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
      0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
      0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
      0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
      0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
      0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
  // rho offsets, lane index x + 5y
  constexpr int ROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
  for (int round = 0; round < 24; round++) {
    uint64_t c[5], b[25];
#pragma unroll
    for (int x = 0; x < 5; x++) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
#pragma unroll
    for (int x = 0; x < 5; x++) {
      const uint64_t d = c[(x + 4) % 5] ^ rotl64(c[(x + 1) % 5], 1);
#pragma unroll
      for (int y = 0; y < 5; y++) a[x + 5 * y] ^= d;
    }
    // rho + pi: B[y, 2x + 3y] = rot(A[x, y])
#pragma unroll
    for (int x = 0; x < 5; x++)
#pragma unroll
      for (int y = 0; y < 5; y++) b[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(a[x + 5 * y], ROT[x + 5 * y]);
    // chi
#pragma unroll
    for (int y = 0; y < 5; y++)
#pragma unroll
      for (int x = 0; x < 5; x++) a[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
    a[0] ^= RC[round];
  }
}

// 32-byte big-endian encoding of a canonical field element as 8 little-endian
// message words (what a byte-wise absorb would read)
DX_HD void be_words(const Fp &v, uint32_t *w) {
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = bswap32(v.v[7 - i]);
}

}  // namespace

extern "C" {
// out[p] = SHA3-512(B || C_p || Y_{cols[p]}) mod r as canonical Fr limbs.
//   C_aff: [n, 16] Montgomery affine commitments (infinity = zeros)
//   b_words: 16 words = B.MarshalBinary() read as little-endian u32
//   y_words: [n_cols, 16] words of the per-column sum_i y_i encodings
int dx_rp_challenges(int on_gpu, void *stream, const uint32_t *C_aff, const uint32_t *b_words,
                     const uint32_t *y_words, const int32_t *cols, uint32_t *out, int64_t n) {
  auto op = [=] __host__ __device__(int64_t p) {
    uint32_t w[48];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = b_words[i];
    const G1A c = at<G1A>(C_aff, p);
    be_words(from_mont(c.x), w + 16);
    be_words(from_mont(c.y), w + 24);
    const uint32_t *yw = y_words + 16 * (int64_t)cols[p];
#pragma unroll
    for (int i = 0; i < 16; i++) w[32 + i] = yw[i];
    // absorb 192 bytes at rate 72 (9 lanes): two full blocks + 48 bytes padded
    uint64_t a[25];
#pragma unroll
    for (int i = 0; i < 25; i++) a[i] = 0;
#pragma unroll
    for (int blk = 0; blk < 3; blk++) {
#pragma unroll
      for (int k = 0; k < 9; k++) {
        const int lane = blk * 9 + k;
        uint64_t v = 0;
        if (lane < 24) v = (uint64_t)w[2 * lane] | ((uint64_t)w[2 * lane + 1] << 32);
        if (lane == 24) v = 0x06ull;                 // SHA-3 domain padding
        if (blk == 2 && k == 8) v ^= 0x8000000000000000ull;
        a[k] ^= v;
      }
      keccak_f1600(a);
    }
    // digest bytes d[0..63] = lanes 0..7 little-endian; x = BE integer of d
    uint32_t dw[16];
#pragma unroll
    for (int m = 0; m < 16; m++) dw[m] = (uint32_t)(a[m >> 1] >> (32 * (m & 1)));
    uint32_t hi[8], lo[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      hi[j] = bswap32(dw[7 - j]);
      lo[j] = bswap32(dw[15 - j]);
    }
    // x mod r = lo + hi * 2^256 = reduce(lo) + mont_mul(reduce(hi), R^2)
    const Fr h = fmul(reduce_256<FrParams>(hi), Fr::from_limbs(FrParams::R2));
    at<Fr>(out, p) = fadd(reduce_256<FrParams>(lo), h);
  };
  return run(on_gpu, stream, n, op, false, "rp_challenges");
}
}
