// K13: logistic-regression approximation-coefficient GEMM on fp64 MFMA.
//
//   out[a][b] = sum_i w[i] * X[i][a] * X[i][b],   X: [N][D] row-major fp64, D <= 48
//
// Reference: lib/encoding/logistic_regression.go:61-111 computes the level-2
// coefficients record by record through cartesian products (O(N (d+1)^2)
// scalar float ops in Go).  Here it is one tall-skinny GEMM over the records:
// K = N is the reduction dimension of v_mfma_f64_16x16x4f64.  For one K-step of
// 4 records, lane l holds X[k][16t + (l&15)] (k = l>>4) for the three 16-column
// tiles t; the same registers are the B operand and, scaled by w[k], the A
// operand, so the 3x3 output tiles need 3 loads + 9 MFMAs per step.  Waves
// stride over records (grid-stride), the 4 waves of a block reduce through LDS
// and each block writes one 48x48 partial; a tiny second pass (torch.sum on the
// [blocks,48,48] slab) finishes deterministically.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef double dx_f64x4 __attribute__((ext_vector_type(4)));

namespace {
constexpr int kTile = 16;
constexpr int kTiles = 3;  // D <= 48
constexpr int kD = kTile * kTiles;
constexpr int kWaves = 4;

__global__ void __launch_bounds__(256) lr_moments_kernel(const double *__restrict__ X, const double *__restrict__ w,
                                                          int64_t N, int D, double *__restrict__ partial) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int col = lane & 15;
  const int kk = lane >> 4;  // 0..3 record within the K-step
  dx_f64x4 acc[kTiles][kTiles];
#pragma unroll
  for (int a = 0; a < kTiles; a++)
#pragma unroll
    for (int b = 0; b < kTiles; b++) acc[a][b] = (dx_f64x4){0.0, 0.0, 0.0, 0.0};

  const int64_t gw = (int64_t)blockIdx.x * kWaves + wave;
  const int64_t nw = (int64_t)gridDim.x * kWaves;
  const int64_t steps = (N + 3) / 4;
  for (int64_t s = gw; s < steps; s += nw) {
    const int64_t row = s * 4 + kk;
    double v[kTiles];
    double wi = 0.0;
    if (row < N) {
      wi = w[row];
      const double *xr = X + row * (int64_t)D;
#pragma unroll
      for (int t = 0; t < kTiles; t++) {
        int c = t * kTile + col;
        v[t] = c < D ? xr[c] : 0.0;
      }
    } else {
#pragma unroll
      for (int t = 0; t < kTiles; t++) v[t] = 0.0;
    }
#pragma unroll
    for (int a = 0; a < kTiles; a++) {
      const double av = v[a] * wi;
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
}  // namespace

extern "C" int dx_lr_moments(void *stream, const double *X, const double *w, int64_t N, int D, double *partial,
                             int n_blocks) {
  if (D > kD || D <= 0) return -2;
  hipLaunchKernelGGL(lr_moments_kernel, dim3(n_blocks), dim3(256), 0, (hipStream_t)stream, X, w, N, D, partial);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    fprintf(stderr, "[drynx_amd native] lr_moments: %s\n", hipGetErrorString(e));
    return -1;
  }
  return 0;
}
