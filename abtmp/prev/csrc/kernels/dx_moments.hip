// K14: exact int64 moments of the DPs' records, all DPs of a rank in one launch.
//
// Every integer encoder of the reference is a handful of sums of products of
// record columns (lib/encoding/sum.go:19-22, mean.go, variance.go:21-24,
// cosim.go:26-34, linear_regression_dims.go:48-89, model_evaluation.go:33-37),
// computed record by record in Go int64 per DP.  Here they are one "augmented
// Gram" reduction: the records of every DP hosted on a rank are stacked into
// one int64 matrix Z [rows][C] (DP g owns rows seg[g]..seg[g+1]), column C is
// a virtual constant 1, and
//
//     out[g][p] = sum_{i in DP g} Z[i][a_p] * Z[i][b_p]      (mod 2^64, like Go)
//
// for a list of column pairs (a_p, b_p) -- (a, C) is sum x_a, (C, C) the record
// count.  Exact integers: VALU 64-bit multiply-adds, never fp MFMA.
//
// GPU: one workgroup per tile (a row range of one DP, planned on the host so
// big DPs are split over many CUs and thousands of one-record DPs are one
// launch).  The tile's rows are staged through LDS 64 at a time with the
// constant column appended; the 256 threads split the (pair, row-lane) space
// (L lanes per pair so that 3 pairs still keep every thread busy), reduce in
// LDS with 64-bit LDS atomics and add one partial per pair to the output with
// a global (vector) 64-bit atomic.  Host path: one partial per tile on the
// thread pool, summed per DP in tile order.
#include "exec.h"

namespace {
constexpr int kRows = 64;
constexpr int kMaxCols = 64;                                   // data columns (+ the constant one)
constexpr int kMaxPairs = (kMaxCols + 1) * (kMaxCols + 2) / 2;  // 2145
constexpr int kThreads = 256;
constexpr int kMaxUnits = (kMaxPairs + kThreads - 1) / kThreads;

struct MomArgs {
  const int64_t *Z;
  int64_t ldz;
  int C;
  const int64_t *tiles;  // [n_tiles][3] = (dp, row0, row1)
  const int16_t *pairs;  // [P][2], column index C = constant 1
  int P;
  int L;  // row lanes per pair
  int64_t *out;  // [n_dp][P], zeroed by the caller
};

__global__ void __launch_bounds__(kThreads) int_moments_kernel(MomArgs a) {
  __shared__ int64_t z[kRows][kMaxCols + 2];
  __shared__ unsigned long long red[kMaxPairs];
  const int64_t dp = a.tiles[3 * blockIdx.x], r0 = a.tiles[3 * blockIdx.x + 1], r1 = a.tiles[3 * blockIdx.x + 2];
  const int W = a.C + 1;
  for (int p = threadIdx.x; p < a.P; p += kThreads) red[p] = 0;

  const int units = a.P * a.L;
  uint64_t acc[kMaxUnits];
  int ca[kMaxUnits], cb[kMaxUnits], lane[kMaxUnits];
#pragma unroll
  for (int k = 0; k < kMaxUnits; k++) {
    const int e = threadIdx.x + k * kThreads;
    acc[k] = 0;
    const int p = e < units ? e / a.L : 0;
    ca[k] = a.pairs[2 * p];
    cb[k] = a.pairs[2 * p + 1];
    lane[k] = e % a.L;
  }

  for (int64_t base = r0; base < r1; base += kRows) {
    const int nr = (int)(r1 - base < kRows ? r1 - base : kRows);
    __syncthreads();
    for (int e = threadIdx.x; e < kRows * W; e += kThreads) {
      const int r = e / W, c = e - r * W;
      z[r][c] = r < nr ? (c < a.C ? a.Z[(base + r) * a.ldz + c] : 1) : 0;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kMaxUnits; k++) {
      if (threadIdx.x + k * kThreads < units) {
        uint64_t s = acc[k];
        for (int r = lane[k]; r < nr; r += a.L) s += (uint64_t)z[r][ca[k]] * (uint64_t)z[r][cb[k]];
        acc[k] = s;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < kMaxUnits; k++) {
    const int e = threadIdx.x + k * kThreads;
    if (e < units && acc[k]) atomicAdd(&red[e / a.L], (unsigned long long)acc[k]);
  }
  __syncthreads();
  for (int p = threadIdx.x; p < a.P; p += kThreads)
    if (red[p]) atomicAdd(reinterpret_cast<unsigned long long *>(a.out + dp * a.P + p), red[p]);
}
}  // namespace

extern "C" int dx_int_moments(int on_gpu, void *stream, const int64_t *Z, int64_t ldz, int C, const int64_t *tiles,
                              int64_t n_tiles, const int16_t *pairs, int P, int64_t *out, int64_t *host_partial) {
  if (C < 0 || C > kMaxCols || P <= 0 || P > kMaxPairs || n_tiles < 0) return -2;
  if (n_tiles == 0) return 0;
  if (on_gpu) {
    int L = 1;
    while (L < kRows && P * L * 2 <= kThreads) L *= 2;
    MomArgs a{Z, ldz, C, tiles, pairs, P, L, out};
    hipLaunchKernelGGL(int_moments_kernel, dim3((unsigned)n_tiles), dim3(kThreads), 0, (hipStream_t)stream, a);
    return dx::check_hip(hipGetLastError(), "int_moments");
  }
  // host: one partial row per tile (parallel), then the per-DP sums in tile order
  dx::host_for_each(n_tiles, [=](int64_t t) {
    const int64_t r0 = tiles[3 * t + 1], r1 = tiles[3 * t + 2];
    uint64_t *row = reinterpret_cast<uint64_t *>(host_partial + t * P);
    for (int p = 0; p < P; p++) row[p] = 0;
    for (int64_t i = r0; i < r1; i++) {
      const int64_t *zi = Z + i * ldz;
      for (int p = 0; p < P; p++) {
        const int ia = pairs[2 * p], ib = pairs[2 * p + 1];
        const uint64_t x = ia < C ? (uint64_t)zi[ia] : 1u, y = ib < C ? (uint64_t)zi[ib] : 1u;
        row[p] += x * y;
      }
    }
  });
  for (int64_t t = 0; t < n_tiles; t++) {
    uint64_t *o = reinterpret_cast<uint64_t *>(out + tiles[3 * t] * P);
    const uint64_t *row = reinterpret_cast<const uint64_t *>(host_partial + t * P);
    for (int p = 0; p < P; p++) o[p] += row[p];
  }
  return 0;
}
