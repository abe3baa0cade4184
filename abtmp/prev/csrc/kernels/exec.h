// Execution helpers: one functor definition per batched op, run either as a
// gfx950 kernel (thread per item, 64-wide waves) on a caller-provided HIP
// stream, or by a host thread pool (CPU parties / CPU test-suite).
#pragma once
#include <hip/hip_runtime.h>
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace dx {

// Every kernel asks for at least 2 waves per SIMD.  The out-of-line tower and
// curve functions are shared by all kernels of a translation unit, and the
// AMDGPU attributor budgets their registers for the least demanding caller:
// without a target on every kernel they may take 256 VGPRs plus up to ~200
// AGPRs, i.e. 1 wave per SIMD, so a 1553-wave range fold ran as one full
// round of 1024 waves and a half-empty second round.  At 2 waves per SIMD
// (256 registers) the extra spills are a few call-frame slots.
#define DX_OCC __attribute__((amdgpu_waves_per_eu(2)))

template <class Op>
__global__ void __launch_bounds__(256) DX_OCC for_each_kernel(int64_t n, Op op) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) op(i);
}

// Heavy per-thread ops (pairings, scalar mults) use 64-thread blocks so many
// workgroups exist even for modest batches (256 CUs want >>256 blocks).
template <class Op>
__global__ void __launch_bounds__(64) DX_OCC for_each_kernel64(int64_t n, Op op) {
  int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (i < n) op(i);
}

inline int host_threads() {
  static int nt = [] {
    const char *e = getenv("DX_NUM_THREADS");
    if (!e) e = getenv("OMP_NUM_THREADS");  // the box's CPU share (16 on a 1-GPU box)
    int v = e ? atoi(e) : (int)std::thread::hardware_concurrency();
    if (v <= 0) v = 1;
    return std::min(v, 32);
  }();
  return nt;
}

// Persistent host worker pool (the host path of every batched op, and the
// short serial tails -- GT product trees, final exponentiations -- that the
// device hands back).  One job at a time; a caller that finds the pool busy
// (another Python thread's op) runs its job inline instead of waiting.
class HostPool {
 public:
  static HostPool &get() {
    static HostPool *p = new HostPool(host_threads() - 1);  // never destroyed: workers outlive static teardown
    return *p;
  }
  // min_par: smallest n worth a dispatch to the workers (heavy per-item ops
  // -- pairings, final exponentiations, GT ladders of a few verifiers -- gain
  // from 2 items on; cheap ones from 4)
  template <class Op>
  void for_each(int64_t n, const Op &op, int64_t min_par = 4) {
    const int64_t chunk = std::max<int64_t>(1, n / ((int64_t)(workers_.size() + 1) * 8));
    std::unique_lock<std::mutex> busy(job_mu_, std::try_to_lock);
    if (!busy.owns_lock() || workers_.empty() || n < min_par) {
      for (int64_t i = 0; i < n; i++) op(i);
      return;
    }
    std::atomic<int64_t> next{0};
    auto body = [&] {
      for (;;) {
        int64_t s = next.fetch_add(chunk);
        if (s >= n) break;
        int64_t e = std::min(n, s + chunk);
        for (int64_t i = s; i < e; i++) op(i);
      }
    };
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = body;
      pending_ = (int)workers_.size();
      gen_++;
    }
    cv_.notify_all();
    body();
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [&] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  explicit HostPool(int n) {
    for (int t = 0; t < n; t++) workers_.emplace_back([this] { loop(); });
    for (auto &w : workers_) w.detach();
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      std::function<void()> job;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return gen_ != seen; });
        seen = gen_;
        job = job_;
      }
      if (job) job();
      {
        std::lock_guard<std::mutex> g(mu_);
        if (--pending_ == 0) done_cv_.notify_all();
      }
    }
  }
  std::vector<std::thread> workers_;
  std::mutex job_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::function<void()> job_;
  uint64_t gen_ = 0;
  int pending_ = 0;
};

template <class Op>
void host_for_each(int64_t n, const Op &op, int64_t min_par = 4) {
  HostPool::get().for_each(n, op, min_par);
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
    host_for_each(n, op, heavy ? 2 : 4);
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
