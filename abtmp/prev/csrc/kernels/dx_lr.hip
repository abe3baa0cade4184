// K13: logistic-regression approximation-coefficient encoder on fp64 MFMA.
//
// One pass over the DP's raw records computes BOTH coefficient levels:
//
//   xa_i      = [1, (X_i - mean) / sd]                (standardise + augment, in registers)
//   out[a][b] = sum_i w_i * xa_i[a] * xa_i[b]          (level 2, w_i = wa*y_i + wb or w[i])
//   out[D][b] = sum_i g_i * xa_i[b],  g_i = 2 y_i - 1  (level 1, in the spare row D)
//
// Reference: lib/encoding/logistic_regression.go:61-111 computes the level-1
// and level-2 coefficients record by record through cartesian products
// (O(N (d+1)^2) scalar float ops in Go, after a separate standardisation pass,
// :367-403).  Here it is one tall-skinny GEMM over the records: K = N is the
// reduction dimension of v_mfma_f64_16x16x4f64.  For one K-step of 4 records,
// lane l holds xa[k][16t + (l&15)] (k = l>>4) for the three 16-column tiles t;
// the same registers are the B operand and, scaled by w[k], the A operand, so
// the 3x3 output tiles need 3 loads + 9 MFMAs per step.  The level-1 vector
// rides in the A operand's spare column D (A = g_i there, B = 0), so it costs
// no extra pass over HBM (it used to be a separate rocBLAS gemv that ran on a
// single workgroup).  Waves stride over records (grid-stride), the 4 waves of
// a block reduce through LDS and each block writes one 48x48 partial; a tiny
// second pass (dx_lr_reduce: fixed summation order over the [blocks,48,48]
// slab, batched over the DPs of a rank) finishes deterministically.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef double dx_f64x4 __attribute__((ext_vector_type(4)));

namespace {
constexpr int kTile = 16;
constexpr int kTiles = 3;  // D <= 48
constexpr int kD = kTile * kTiles;
constexpr int kWaves = 4;

struct LrArgs {
  const double *X;     // [N][dx], row stride ldx
  int64_t ldx;
  int64_t N;
  int dx;              // raw feature columns
  int aug;             // 1: prepend the constant-1 column
  const double *mean;  // [dx] or null (no standardisation)
  const double *sd;    // [dx] or null
  const double *w;     // [N] per-record level-2 weight, or null -> wa*y + wb
  const double *y;     // [N] labels (double) or null
  double wa, wb;
  int level1;          // 1: g = 2y - 1 accumulated in row D
};

__global__ void __launch_bounds__(256) lr_encode_kernel(LrArgs p, double *__restrict__ partial) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int col = lane & 15;
  const int kk = lane >> 4;  // 0..3 record within the K-step
  const int D = p.dx + p.aug;
  dx_f64x4 acc[kTiles][kTiles];
#pragma unroll
  for (int a = 0; a < kTiles; a++)
#pragma unroll
    for (int b = 0; b < kTiles; b++) acc[a][b] = (dx_f64x4){0.0, 0.0, 0.0, 0.0};

  // per-lane standardisation constants of the three columns this lane owns
  double mu[kTiles], sdv[kTiles];
  int src[kTiles];
#pragma unroll
  for (int t = 0; t < kTiles; t++) {
    const int c = t * kTile + col;
    src[t] = c - p.aug;  // raw column, -1 for the augmentation column
    const bool raw = (c < D) && src[t] >= 0;
    mu[t] = (raw && p.mean) ? p.mean[src[t]] : 0.0;
    sdv[t] = (raw && p.sd) ? p.sd[src[t]] : 1.0;
  }

  const int64_t gw = (int64_t)blockIdx.x * kWaves + wave;
  const int64_t nw = (int64_t)gridDim.x * kWaves;
  const int64_t steps = (p.N + 3) / 4;
  for (int64_t s = gw; s < steps; s += nw) {
    const int64_t row = s * 4 + kk;
    double v[kTiles];
    double wi = 0.0, gi = 0.0;
    if (row < p.N) {
      const double yi = p.y ? p.y[row] : 0.0;
      wi = p.w ? p.w[row] : p.wa * yi + p.wb;
      gi = 2.0 * yi - 1.0;
      const double *xr = p.X + row * p.ldx;
#pragma unroll
      for (int t = 0; t < kTiles; t++) {
        const int c = t * kTile + col;
        if (c >= D) v[t] = 0.0;
        else if (src[t] < 0) v[t] = 1.0;
        else v[t] = (xr[src[t]] - mu[t]) / sdv[t];
      }
    } else {
#pragma unroll
      for (int t = 0; t < kTiles; t++) v[t] = 0.0;
    }
#pragma unroll
    for (int a = 0; a < kTiles; a++) {
      const int c = a * kTile + col;
      const double av = (p.level1 && c == D) ? gi : v[a] * wi;
#pragma unroll
      for (int b = 0; b < kTiles; b++) acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, v[b], acc[a][b], 0, 0, 0);
    }
  }

  // f64 16x16x4 C layout: col = lane & 15, row = (lane >> 4) + 4 * reg
  __shared__ double red[kWaves][kD][kD];
#pragma unroll
  for (int a = 0; a < kTiles; a++)
#pragma unroll
    for (int b = 0; b < kTiles; b++)
#pragma unroll
      for (int r = 0; r < 4; r++) red[wave][a * kTile + kk + 4 * r][b * kTile + col] = acc[a][b][r];
  __syncthreads();
  double *out = partial + (int64_t)blockIdx.x * kD * kD;
  for (int e = threadIdx.x; e < kD * kD; e += blockDim.x) {
    const int i = e / kD, j = e % kD;
    out[e] = red[0][i][j] + red[1][i][j] + red[2][i][j] + red[3][i][j];
  }
}

int launch(void *stream, const LrArgs &a, double *partial, int n_blocks) {
  const int D = a.dx + a.aug;
  if (a.dx <= 0 || D > kD || (a.level1 && D >= kD) || n_blocks <= 0) return -2;
  if ((a.level1 || !a.w) && !a.y) return -2;
  hipLaunchKernelGGL(lr_encode_kernel, dim3(n_blocks), dim3(256), 0, (hipStream_t)stream, a, partial);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    fprintf(stderr, "[drynx_amd native] lr_encode: %s\n", hipGetErrorString(e));
    return -1;
  }
  return 0;
}
}  // namespace

// sum_i w_i X_i X_i^T over already-prepared rows (no standardisation, no level 1).
extern "C" int dx_lr_moments(void *stream, const double *X, const double *w, int64_t N, int D, double *partial,
                             int n_blocks) {
  LrArgs a{X, D, N, D, 0, nullptr, nullptr, w, nullptr, 0.0, 0.0, 0};
  return launch(stream, a, partial, n_blocks);
}

// Block partials -> totals, for many encoder launches at once: out[i][e] =
// sum_b partial[i][b][e] in a fixed order (block b into accumulator b % 4,
// then combined), so a DP's coefficients are the same bits whether its
// partials are reduced alone or with the other DPs of its rank.  One thread
// per (item, element): consecutive threads read consecutive elements.
namespace {
__global__ void __launch_bounds__(256) lr_reduce_kernel(const double *__restrict__ partial, int64_t nb, int64_t n_el,
                                                        int64_t n_items, double *__restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_items * n_el) return;
  const int64_t i = t / n_el, e = t % n_el;
  const double *p = partial + i * nb * n_el + e;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  int64_t b = 0;
  for (; b + 4 <= nb; b += 4) {
    s0 += p[(b + 0) * n_el];
    s1 += p[(b + 1) * n_el];
    s2 += p[(b + 2) * n_el];
    s3 += p[(b + 3) * n_el];
  }
  // block b always lands in accumulator b % 4: trailing all-zero blocks (a
  // shorter DP in a batch padded to the longest) leave the sums unchanged
  if (b < nb) s0 += p[b * n_el];
  if (b + 1 < nb) s1 += p[(b + 1) * n_el];
  if (b + 2 < nb) s2 += p[(b + 2) * n_el];
  out[t] = (s0 + s1) + (s2 + s3);
}
}  // namespace

extern "C" int dx_lr_reduce(void *stream, const double *partial, int64_t nb, int64_t n_el, int64_t n_items,
                            double *out) {
  const int64_t n = n_items * n_el;
  if (n <= 0 || nb <= 0) return -2;
  hipLaunchKernelGGL(lr_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, partial,
                     nb, n_el, n_items, out);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    fprintf(stderr, "[drynx_amd native] lr_reduce: %s\n", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

// Fused DP encoder: standardise + augment + level-1 (row D) + level-2 ((wa*y + wb) weights).
extern "C" int dx_lr_encode(void *stream, const double *X, int64_t ldx, int64_t N, int dx, const double *mean,
                            const double *sd, const double *y, double wa, double wb, double *partial, int n_blocks) {
  LrArgs a{X, ldx, N, dx, 1, mean, sd, nullptr, y, wa, wb, 1};
  return launch(stream, a, partial, n_blocks);
}

// Querier gradient descent for k = 2 (FindMinimumWeights, reference
// lib/encoding/logistic_regression.go:693-742; the Cost accumulation quirk and
// the "last weights with Cost >= 0" rule kept): one (d+1)x(d+1) mat-vec per
// iteration with S = A2 + A2^T, on the host.  Runs outside the Python GIL (a
// numpy loop of 450 iterations held it for ~2.6 ms beside the VN checks).
extern "C" int dx_lr_gd_k2(const double *a0, const double *S, const double *w0, int d1, double N, double lam,
                           double step, int max_iter, double C0, double C1, double C2, double *min_w) {
  std::vector<double> w(w0, w0 + d1), Sw(d1), g(d1);
  for (int i = 0; i < d1; i++) min_w[i] = w[i];
  for (int it = 0; it < max_iter; it++) {
    double wa = 0.0, wsw = 0.0, reg = 0.0;
    for (int i = 0; i < d1; i++) {
      double acc = 0.0;
      for (int j = 0; j < d1; j++) acc += S[(int64_t)i * d1 + j] * w[j];
      Sw[i] = acc;
    }
    for (int i = 0; i < d1; i++) {
      wa += w[i] * a0[i];
      wsw += w[i] * Sw[i];
      if (i) reg += w[i] * w[i];
    }
    double c = (wa * C1 + 0.5 * wsw) * C2;
    c = c / N - C0 + (lam / (2 * N)) * reg;
    if (c >= 0.0)
      for (int i = 0; i < d1; i++) min_w[i] = w[i];
    for (int i = 0; i < d1; i++) {
      g[i] = (C1 * a0[i] + C2 * Sw[i]) / N + (i ? (lam / N) * w[i] : 0.0);
      w[i] = w[i] - step * g[i];
    }
  }
  return 0;
}
