// Data-movement glue of the verifier in single launches sized for 256 CUs.
//
//  * dx_batched_copy: many (src, dst, words) regions -- every field of every
//    request's proof list into the batch's columnar arrays (rp.rpl_cat), a
//    VN's list stacked behind its Frobenius image, ... -- in ONE launch of
//    16 KB chunks (one 256-thread workgroup each, 16 dword loads in flight
//    per lane).  torch.cat of a few large contiguous tensors launched ~50
//    workgroups on this image (CatArrayBatchedCopy: ~55 GB/s, 10 ms per
//    query-sized cat in the kernel trace, profiles/r4/kernel_cost_*).
//  * dx_rows_all: the per-proof AND of up to kMaxFlags validity arrays (each
//    uint8 [n * k_i], proof-major) -- one wavefront per proof, a wave-wide
//    vote; replaces the bool conversions + reductions of validate_list.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>

#include "exec.h"

namespace {

constexpr int kChunkWords = 4096;  // 16 KB per workgroup
constexpr int kPerLane = kChunkWords / 256;
constexpr int kMaxFlags = 16;

struct CopyDesc {
  const uint32_t *src;
  uint32_t *dst;
  int64_t words;
  int64_t chunk0;  // first chunk of this region (exclusive prefix sum)
};

__global__ void __launch_bounds__(256) batched_copy_kernel(const CopyDesc *__restrict__ d, int nd) {
  const int64_t c = blockIdx.x;
  int lo = 0, hi = nd - 1;
  while (lo < hi) {  // last region with chunk0 <= c
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].chunk0 <= c) lo = mid; else hi = mid - 1;
  }
  const uint32_t *__restrict__ src = d[lo].src;
  uint32_t *__restrict__ dst = d[lo].dst;
  const int64_t base = (c - d[lo].chunk0) * kChunkWords;
  const int64_t rem = d[lo].words - base;
  const int lim = rem < kChunkWords ? (int)rem : kChunkWords;
  uint32_t v[kPerLane];
#pragma unroll
  for (int k = 0; k < kPerLane; k++) {
    const int i = threadIdx.x + k * 256;
    if (i < lim) v[k] = src[base + i];
  }
#pragma unroll
  for (int k = 0; k < kPerLane; k++) {
    const int i = threadIdx.x + k * 256;
    if (i < lim) dst[base + i] = v[k];
  }
}

// The ledger's device-to-host copy of a query's payloads (~540 MB) straight
// into pinned host memory by a SMALL persistent grid: every block walks the
// chunks c = blockIdx.x, blockIdx.x + gridDim.x, ...  The copy is PCIe-bound
// either way; the runtime's blit kernel ran it on ~4096 waves that held their
// CU slots while stalled on PCIe, beside the verification kernels (5 ms of the
// headline, tools/ab_ledger_copy.py); a 32-block grid leaves them the chip.
__global__ void __launch_bounds__(256) copy_out_kernel(const CopyDesc *__restrict__ d, int nd, int64_t chunks) {
  for (int64_t c = blockIdx.x; c < chunks; c += gridDim.x) {
    int lo = 0, hi = nd - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (d[mid].chunk0 <= c) lo = mid; else hi = mid - 1;
    }
    const uint32_t *__restrict__ src = d[lo].src;
    uint32_t *__restrict__ dst = d[lo].dst;
    const int64_t base = (c - d[lo].chunk0) * kChunkWords;
    const int64_t rem = d[lo].words - base;
    const int lim = rem < kChunkWords ? (int)rem : kChunkWords;
    uint32_t v[kPerLane];
#pragma unroll
    for (int k = 0; k < kPerLane; k++) {
      const int i = threadIdx.x + k * 256;
      if (i < lim) v[k] = src[base + i];
    }
#pragma unroll
    for (int k = 0; k < kPerLane; k++) {
      const int i = threadIdx.x + k * 256;
      if (i < lim) dst[base + i] = v[k];
    }
  }
}

struct FlagSet {
  const uint8_t *f[kMaxFlags];
  int64_t k[kMaxFlags];
  int nf;
};

// one 64-lane wavefront per proof (4 per workgroup)
__global__ void __launch_bounds__(256) rows_all_kernel(FlagSet fs, int64_t n, uint8_t *out) {
  const int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (p >= n) return;
  int ok = 1;
  for (int a = 0; a < fs.nf; a++) {
    const int64_t k = fs.k[a];
    const uint8_t *row = fs.f[a] + p * k;
    for (int64_t j = lane; j < k; j += 64) ok &= row[j] != 0;
  }
  ok = __all(ok);
  if (lane == 0) out[p] = (uint8_t)(ok ? 1 : 0);
}

}  // namespace

extern "C" {

// desc: [nd, 4] int64 rows (src address, dst address, words, first chunk),
// host-readable copy in desc_host (the CPU path), device copy in desc_dev
int dx_batched_copy(int on_gpu, void *stream, const int64_t *desc_dev, const int64_t *desc_host, int nd,
                    int64_t chunks) {
  if (nd <= 0 || chunks <= 0) return 0;
  if (!on_gpu) {
    dx::host_for_each(nd, [&](int64_t i) {
      const int64_t *e = desc_host + 4 * i;
      std::memcpy(reinterpret_cast<void *>(e[1]), reinterpret_cast<const void *>(e[0]), (size_t)e[2] * 4);
    });
    return 0;
  }
  hipLaunchKernelGGL(batched_copy_kernel, dim3((unsigned)chunks), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const CopyDesc *>(desc_dev), nd);
  return dx::check_hip(hipGetLastError(), "batched_copy");
}

// the same descriptors, dst in pinned host memory (device-visible addresses
// from dx_host_device_ptr), copied by a grid of `blocks` workgroups
int dx_copy_out(int on_gpu, void *stream, const int64_t *desc_dev, const int64_t *desc_host, int nd, int64_t chunks,
                int blocks) {
  if (nd <= 0 || chunks <= 0) return 0;
  if (!on_gpu) return dx_batched_copy(0, stream, desc_dev, desc_host, nd, chunks);
  const unsigned g = (unsigned)(blocks < 1 ? 1 : (chunks < blocks ? chunks : blocks));
  hipLaunchKernelGGL(copy_out_kernel, dim3(g), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const CopyDesc *>(desc_dev), nd, chunks);
  return dx::check_hip(hipGetLastError(), "copy_out");
}

// device-visible address of pinned (hipHostMalloc'd) host memory
int dx_host_device_ptr(void *host, int64_t *out) {
  void *d = nullptr;
  if (dx::check_hip(hipHostGetDevicePointer(&d, host, 0), "hipHostGetDevicePointer")) return -1;
  *out = reinterpret_cast<int64_t>(d);
  return 0;
}

// out[p] = AND over the nf arrays a of all(flags_a[p*k_a : (p+1)*k_a] != 0)
int dx_rows_all(int on_gpu, void *stream, const int64_t *ptrs, const int64_t *ks, int nf, int64_t n, uint8_t *out) {
  if (n <= 0) return 0;
  if (nf > kMaxFlags || nf < 0) return -1;
  FlagSet fs{};
  fs.nf = nf;
  for (int a = 0; a < nf; a++) {
    fs.f[a] = reinterpret_cast<const uint8_t *>(ptrs[a]);
    fs.k[a] = ks[a];
  }
  if (!on_gpu) {
    dx::host_for_each(n, [&](int64_t p) {
      int ok = 1;
      for (int a = 0; a < fs.nf; a++)
        for (int64_t j = 0; j < fs.k[a]; j++) ok &= fs.f[a][p * fs.k[a] + j] != 0;
      out[p] = (uint8_t)ok;
    });
    return 0;
  }
  hipLaunchKernelGGL(rows_all_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, fs, n, out);
  return dx::check_hip(hipGetLastError(), "rows_all");
}

}  // extern "C"
