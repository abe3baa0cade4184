// Execution helpers: one functor definition per batched op, run either as a
// gfx950 kernel (thread per item, 64-wide waves) on a caller-provided HIP
// stream, or by a host thread pool (CPU parties / CPU test-suite).
#pragma once
#include <hip/hip_runtime.h>
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <thread>
#include <vector>

namespace dx {

template <class Op>
__global__ void __launch_bounds__(256) for_each_kernel(int64_t n, Op op) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) op(i);
}

// Heavy per-thread ops (pairings, scalar mults) use 64-thread blocks so many
// workgroups exist even for modest batches (256 CUs want >>256 blocks).
template <class Op>
__global__ void __launch_bounds__(64) for_each_kernel64(int64_t n, Op op) {
  int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (i < n) op(i);
}

inline int host_threads() {
  static int nt = [] {
    const char *e = getenv("DX_NUM_THREADS");
    int v = e ? atoi(e) : (int)std::thread::hardware_concurrency();
    if (v <= 0) v = 1;
    return std::min(v, 64);
  }();
  return nt;
}

template <class Op>
void host_for_each(int64_t n, const Op &op) {
  int nt = host_threads();
  if (n < 2 || nt == 1) {
    for (int64_t i = 0; i < n; i++) op(i);
    return;
  }
  std::atomic<int64_t> next{0};
  const int64_t chunk = std::max<int64_t>(1, n / (nt * 8));
  auto worker = [&] {
    for (;;) {
      int64_t s = next.fetch_add(chunk);
      if (s >= n) break;
      int64_t e = std::min(n, s + chunk);
      for (int64_t i = s; i < e; i++) op(i);
    }
  };
  std::vector<std::thread> th;
  int use = (int)std::min<int64_t>(nt, (n + chunk - 1) / chunk);
  for (int t = 1; t < use; t++) th.emplace_back(worker);
  worker();
  for (auto &t : th) t.join();
}

inline int check_hip(hipError_t e, const char *what) {
  if (e != hipSuccess) {
    fprintf(stderr, "[drynx_amd native] HIP error in %s: %s\n", what, hipGetErrorString(e));
    return -1;
  }
  return 0;
}

// Run op over [0,n): on_gpu selects the device path on `stream`.
template <class Op>
int run(int on_gpu, void *stream, int64_t n, const Op &op, bool heavy = false, const char *name = "op") {
  if (n <= 0) return 0;
  if (!on_gpu) {
    host_for_each(n, op);
    return 0;
  }
  hipStream_t s = (hipStream_t)stream;
  if (heavy) {
    int64_t blocks = (n + 63) / 64;
    hipLaunchKernelGGL(for_each_kernel64<Op>, dim3((unsigned)blocks), dim3(64), 0, s, n, op);
  } else {
    int64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(for_each_kernel<Op>, dim3((unsigned)blocks), dim3(256), 0, s, n, op);
  }
  return check_hip(hipGetLastError(), name);
}

}  // namespace dx
