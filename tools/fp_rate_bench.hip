// Microbenchmark: issue rates of the instructions a BN254 field multiplication
// can be built from on gfx950, and the production Montgomery multiply
// (csrc/bn254/field.h fmul) itself -- to price a 52-bit-limb FP64 FMA field
// (Emmart-Zheng-Weems style: exact products split by two FMAs) against the
// 32-bit-limb integer path.  Every kernel runs 8 independent chains per lane
// (enough ILP to measure issue rate, not latency) over a full-chip grid.
//
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I csrc tools/fp_rate_bench.hip -o tools/bin/fp_rate_bench
// Run:   tools/bin/fp_rate_bench
#define DX_NI __host__ __device__ __forceinline__
#include "kernels/common.h"

#include <chrono>
#include <cstdio>
#include <vector>

namespace {
constexpr int kWG = 256;
constexpr int kChains = 8;

__global__ void __launch_bounds__(kWG) mad_u64_kernel(uint64_t *out, int iters) {
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  uint64_t acc[kChains];
  uint32_t a = (uint32_t)i * 2654435761u + 1u, b = (uint32_t)i ^ 0x9e3779b9u;
#pragma unroll
  for (int c = 0; c < kChains; c++) acc[c] = (uint64_t)c * 7919u + i;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < kChains; c++) acc[c] = (uint64_t)(uint32_t)acc[c] * (a + c) + (acc[c] >> 32) + b;
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < kChains; c++) s ^= acc[c];
  out[i] = s;
}

__global__ void __launch_bounds__(kWG) mul_lo_hi_kernel(uint32_t *out, int iters) {
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  uint32_t lo[kChains], hi[kChains];
  const uint32_t a = (uint32_t)i * 2654435761u + 1u;
#pragma unroll
  for (int c = 0; c < kChains; c++) {
    lo[c] = (uint32_t)(c * 7919 + i);
    hi[c] = (uint32_t)(c * 31 + i);
  }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < kChains; c++) {
      const uint32_t l = lo[c] * (a + c), h = __umulhi(hi[c], a + c);
      lo[c] = l ^ h;
      hi[c] = h + l;
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < kChains; c++) s ^= lo[c] ^ hi[c];
  out[i] = s;
}

__global__ void __launch_bounds__(kWG) fma_f64_kernel(double *out, int iters) {
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  double acc[kChains];
  const double a = 1.0000001 + 1e-12 * (double)(i & 1023), b = 1e-9;
#pragma unroll
  for (int c = 0; c < kChains; c++) acc[c] = 1.0 + c;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < kChains; c++) acc[c] = fma(acc[c], a, b);
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < kChains; c++) s += acc[c];
  out[i] = s;
}

__global__ void __launch_bounds__(kWG) fma_f32_kernel(float *out, int iters) {
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  float acc[kChains];
  const float a = 1.0000001f, b = 1e-9f;
#pragma unroll
  for (int c = 0; c < kChains; c++) acc[c] = 1.0f + c + (float)(i & 7);
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < kChains; c++) acc[c] = fmaf(acc[c], a, b);
  }
  float s = 0;
#pragma unroll
  for (int c = 0; c < kChains; c++) s += acc[c];
  out[i] = s;
}

// production Montgomery multiply: 4 independent chains (each an 8-limb Fp)
__global__ void __launch_bounds__(kWG) DX_OCC fmul_kernel(const uint32_t *in, uint32_t *out, int iters) {
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  Fp x[4], y = at<Fp>(in, 4);
#pragma unroll
  for (int c = 0; c < 4; c++) x[c] = at<Fp>(in, c);
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < 4; c++) x[c] = fmul(x[c], y);
  }
  Fp s = x[0];
#pragma unroll
  for (int c = 1; c < 4; c++) s = fadd(s, x[c]);
  at<Fp>(out, i) = s;
}

template <class F>
double time_ms(F &&launch) {
  launch();
  (void)hipDeviceSynchronize();
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < 3; r++) launch();
  (void)hipDeviceSynchronize();
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / 3;
}
}  // namespace

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const int64_t blocks = (int64_t)cus * 8;  // 8 waves of 256 lanes... 2048 lanes per CU
  const int64_t n = blocks * kWG;
  const int iters = 4096;
  void *buf;
  (void)hipMalloc(&buf, n * 64);
  std::vector<uint32_t> h(5 * 8);
  for (int k = 0; k < 5; k++) {  // small canonical Montgomery-form values
    for (int l = 0; l < 8; l++) h[k * 8 + l] = l < 7 ? 0x12345678u * (k + 1) + l : 0x01000000u;
  }
  uint32_t *in;
  (void)hipMalloc(&in, h.size() * 4);
  (void)hipMemcpy(in, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  const double ops = (double)n * iters * kChains;
  double ms;
  ms = time_ms([&] { hipLaunchKernelGGL(mad_u64_kernel, dim3(blocks), dim3(kWG), 0, 0, (uint64_t *)buf, iters); });
  printf("v_mad_u64_u32 chains   : %8.3f ms  %8.1f G ops/s  %6.1f lane-ops/clk/CU (at %d MHz)\n", ms, ops / ms / 1e6,
         ops / (ms * 1e-3) / cus / (prop.clockRate * 1e3), prop.clockRate / 1000);
  ms = time_ms([&] { hipLaunchKernelGGL(mul_lo_hi_kernel, dim3(blocks), dim3(kWG), 0, 0, (uint32_t *)buf, iters); });
  printf("mul_lo + mul_hi u32    : %8.3f ms  %8.1f G pairs/s %6.1f pairs/clk/CU\n", ms, ops / ms / 1e6,
         ops / (ms * 1e-3) / cus / (prop.clockRate * 1e3));
  ms = time_ms([&] { hipLaunchKernelGGL(fma_f64_kernel, dim3(blocks), dim3(kWG), 0, 0, (double *)buf, iters); });
  printf("v_fma_f64              : %8.3f ms  %8.1f G ops/s  %6.1f lane-ops/clk/CU\n", ms, ops / ms / 1e6,
         ops / (ms * 1e-3) / cus / (prop.clockRate * 1e3));
  ms = time_ms([&] { hipLaunchKernelGGL(fma_f32_kernel, dim3(blocks), dim3(kWG), 0, 0, (float *)buf, iters); });
  printf("v_fma_f32              : %8.3f ms  %8.1f G ops/s  %6.1f lane-ops/clk/CU\n", ms, ops / ms / 1e6,
         ops / (ms * 1e-3) / cus / (prop.clockRate * 1e3));
  const int fiters = 512;
  const double fops = (double)n * fiters * 4;
  ms = time_ms([&] { hipLaunchKernelGGL(fmul_kernel, dim3(blocks), dim3(kWG), 0, 0, in, (uint32_t *)buf, fiters); });
  printf("Fp fmul (field.h)      : %8.3f ms  %8.2f G fmul/s  %6.3f fmul/clk/CU\n", ms, fops / ms / 1e6,
         fops / (ms * 1e-3) / cus / (prop.clockRate * 1e3));
  (void)hipFree(buf);
  (void)hipFree(in);
  return 0;
}
