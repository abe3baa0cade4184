// Microbenchmark: chains of GT (Fp12) products f <- f * T[e] (or * conj(T[e])),
// the inner loop of the range prover (prove_e / prove_t) and of the verifier's
// GT bucket accumulation (gt_slice_prod).
//
//   A: one lane per item (the production layout up to round 3): the whole
//      Fp12 accumulator, the operand and the Karatsuba temporaries live in
//      one lane -- ~700 registers of working set, scratch spills at 2 waves
//      per SIMD.
//   B: three lanes per item.  Fp12 = a0 + a1 w over Fp6; Karatsuba needs
//      t0 = a0 b0, t1 = a1 b1, t2 = (a0 + a1)(b0 + b1): lane r of the triple
//      holds role r's Fp6 pair and computes ONE Fp6 product; the outputs
//        c0 = t0 + v t1,  c1 = t2 - t0 - t1,  c0 + c1 = t2 + (v - 1) t1
//      are formed after two 48-dword lane shuffles (ds_bpermute), so every
//      lane ends the step holding its role's operand for the next product.
//
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I csrc tools/fp12_coop_bench.hip -o build/fp12_coop_bench
// Run:   build/fp12_coop_bench [items] [products] [table_entries]
#define DX_NI __host__ __device__ __forceinline__
#include "kernels/common.h"

#include <chrono>
#include <random>
#include <vector>

namespace {
constexpr int kWG = 64;
constexpr int kPer = kWG / 3;  // 21 items per 64-lane wave (lane 63 idle)

__global__ void __launch_bounds__(kWG) DX_OCC chain_a(const Fp12 *T, const uint32_t *idx, Fp12 *out, int64_t n, int K) {
  const int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (i >= n) return;
  Fp12 f = Fp12::one();
  for (int k = 0; k < K; k++) {
    const uint32_t e = idx[i * K + k];
    const Fp12 &b = T[e >> 1];
    f = mul(f, (e & 1) ? conj(b) : b);
  }
  out[i] = f;
}

DX_HD Fp6 sel6(bool c, const Fp6 &a, const Fp6 &b) {
  Fp6 r;
  const uint32_t *pa = &a.c0.c0.v[0], *pb = &b.c0.c0.v[0];
  uint32_t *pr = &r.c0.c0.v[0];
#pragma unroll
  for (int i = 0; i < 48; i++) pr[i] = c ? pa[i] : pb[i];
  return r;
}

__device__ __forceinline__ Fp6 shfl6(const Fp6 &a, int src) {
  Fp6 r;
  const uint32_t *pa = &a.c0.c0.v[0];
  uint32_t *pr = &r.c0.c0.v[0];
#pragma unroll
  for (int i = 0; i < 48; i++) pr[i] = (uint32_t)__shfl((int)pa[i], src, 64);
  return r;
}

__device__ __forceinline__ Fp6 load6(const Fp6 *p) { return *p; }

template <int WAVES>
__global__ void __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(WAVES))) chain_b(const Fp12 *T,
    const uint32_t *idx, Fp12 *out, int64_t n, int K) {
  const int lane = threadIdx.x;
  const int g = lane / 3, r = lane - 3 * g;
  const int base = 3 * g;
  const int64_t i = (int64_t)blockIdx.x * kPer + g;
  const bool live = g < kPer && i < n;
  // f = 1: a0 = 1, a1 = 0, a0 + a1 = 1
  Fp6 x = r == 1 ? Fp6::zero() : Fp6::one();
  for (int k = 0; k < K; k++) {
    const uint32_t e = live ? idx[i * K + k] : 0u;
    const Fp12 *b = T + (e >> 1);
    // role operand: r0 b0, r1 +-b1, r2 b0 +- b1 (conj: b1 -> -b1)
    const Fp6 y0 = r != 1 ? load6(&b->c0) : Fp6::zero();
    const Fp6 y1 = r != 0 ? load6(&b->c1) : Fp6::zero();
    const Fp6 y = (e & 1) ? sub(y0, y1) : add(y0, y1);
    const Fp6 t = mul(x, y);
    const Fp6 p = shfl6(t, base + (r == 1 ? 0 : 1));  // r0, r2: t1 ; r1: t0
    const Fp6 q = shfl6(t, base + 2);                 // r1: t2
    const Fp6 u = add(t, mul_v(p));                   // r0: c0 ; r2: t2 + v t1
    // r0: u ; r1: t2 - t0 - t1 ; r2: u - t1
    x = sub(sub(sel6(r == 1, q, u), sel6(r == 0, Fp6::zero(), p)), sel6(r == 1, t, Fp6::zero()));
  }
  if (live && r < 2) {
    Fp6 *o = r == 0 ? &out[i].c0 : &out[i].c1;
    *o = x;
  }
}
}  // namespace

static void check(hipError_t e, const char *w) {
  if (e != hipSuccess) {
    fprintf(stderr, "%s: %s\n", w, hipGetErrorString(e));
    exit(1);
  }
}

int main(int argc, char **argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 993600;
  const int K = argc > 2 ? atoi(argv[2]) : 34;
  const int64_t nt = argc > 3 ? atoll(argv[3]) : (1 << 20);
  std::mt19937_64 rng(7);
  std::vector<Fp12> T(nt);
  for (auto &t : T) {
    uint32_t *p = &t.c0.c0.c0.v[0];
    for (int i = 0; i < 96; i++) p[i] = (uint32_t)rng();
    for (int c = 0; c < 12; c++) p[8 * c + 7] &= 0x0fffffffu;  // < p
  }
  std::vector<uint32_t> idx((size_t)n * K);
  for (auto &v : idx) v = (uint32_t)(rng() % (uint64_t)(2 * nt));
  Fp12 *dT, *dA, *dB;
  uint32_t *dI;
  check(hipMalloc(&dT, nt * sizeof(Fp12)), "malloc");
  check(hipMalloc(&dA, n * sizeof(Fp12)), "malloc");
  check(hipMalloc(&dB, n * sizeof(Fp12)), "malloc");
  check(hipMalloc(&dI, idx.size() * 4), "malloc");
  check(hipMemcpy(dT, T.data(), nt * sizeof(Fp12), hipMemcpyHostToDevice), "h2d");
  check(hipMemcpy(dI, idx.data(), idx.size() * 4, hipMemcpyHostToDevice), "h2d");
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const dim3 ga((unsigned)((n + kWG - 1) / kWG)), gb((unsigned)((n + kPer - 1) / kPer));
  for (int variant = 0; variant < 4; variant++) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; rep++) {
      hipEventRecord(e0);
      if (variant == 0)
        hipLaunchKernelGGL(chain_a, ga, dim3(kWG), 0, 0, dT, dI, dA, n, K);
      else if (variant == 1)
        hipLaunchKernelGGL(chain_b<2>, gb, dim3(kWG), 0, 0, dT, dI, dB, n, K);
      else if (variant == 2)
        hipLaunchKernelGGL(chain_b<3>, gb, dim3(kWG), 0, 0, dT, dI, dB, n, K);
      else
        hipLaunchKernelGGL(chain_b<4>, gb, dim3(kWG), 0, 0, dT, dI, dB, n, K);
      hipEventRecord(e1);
      check(hipEventSynchronize(e1), "sync");
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    printf("{\"variant\": \"%s\", \"items\": %lld, \"products\": %d, \"table\": %lld, \"ms\": %.3f, "
           "\"Mmul_per_s\": %.1f}\n",
           variant == 0 ? "A_one_lane" : variant == 1 ? "B3_w2" : variant == 2 ? "B3_w3" : "B3_w4", (long long)n, K, (long long)nt, best,
           (double)n * K / best / 1e3);
    fflush(stdout);
  }
  std::vector<Fp12> a(n), b(n);
  check(hipMemcpy(a.data(), dA, n * sizeof(Fp12), hipMemcpyDeviceToHost), "d2h");
  check(hipMemcpy(b.data(), dB, n * sizeof(Fp12), hipMemcpyDeviceToHost), "d2h");
  int64_t bad = 0;
  for (int64_t i = 0; i < n; i++) bad += !(a[i] == b[i]);
  printf("{\"mismatches\": %lld}\n", (long long)bad);
  return bad ? 2 : 0;
}
