// Bucket plans of the Pippenger MSMs / multi-exponentiations (G1, G2, GT):
// the (group, window, digit) keys of every scalar entry are sorted with their
// entry index, then every non-empty bucket is cut into slices of <= sl
// entries that one thread reduces per pass.
//
//  * dx_bucket_sort: rocPRIM radix sort of (key, item) pairs over the low
//    end_bit bits only (the keys of a plan are < 2^end_bit; the zero-digit
//    sentinel 0x7fffffff has all of those bits set, so it sorts last), 4-byte
//    payload -- instead of a full 32-bit sort with an 8-byte index payload
//    and a gather of the items.
//  * dx_bucket_bounds: first entry and end of every bucket's run in the sorted
//    keys (run boundaries only: coalesced reads, one write per boundary).
//  * dx_bucket_hist + dx_bucket_scatter: a counting sort by bucket (the keys
//    are small integers): one histogram pass, one scatter pass -- no
//    comparison / radix sort, no index payload, no gather; the histogram is
//    the plan's per-bucket counts.
//  * dx_slice_desc: one thread per slice (binary search of its bucket)
//    writes the pass descriptors (start, length), coalesced -- they never go
//    through torch's repeat_interleave / arange / index arithmetic.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <rocprim/device/device_radix_sort.hpp>
#include <vector>

#include "exec.h"

namespace {

__global__ void __launch_bounds__(256) bucket_bounds_kernel(const int32_t *keys, int64_t n, int64_t nb,
                                                            int64_t *first, int64_t *end) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int32_t k = keys[i];
  if (k < 0 || k >= nb) return;  // zero-digit sentinel
  if (i == 0 || keys[i - 1] != k) first[k] = i;
  if (i + 1 == n || keys[i + 1] != k) end[k] = i + 1;
}

__global__ void __launch_bounds__(256) slice_plan_kernel(const int64_t *first, const int64_t *count,
                                                         const int64_t *soff, int sl, int64_t nbk, int64_t *st,
                                                         int32_t *ln) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= nbk) return;
  const int64_t c = count[b], f = first[b], o = soff[b];
  const int64_t ns = (c + sl - 1) / sl;
  for (int64_t j = 0; j < ns; j++) {
    st[o + j] = f + j * sl;
    ln[o + j] = (int32_t)std::min<int64_t>(sl, c - j * sl);
  }
}

// counting sort of the entries by bucket: histogram, then each entry's slot
// = offs[key] + (arrival order within its bucket); the order inside a bucket
// is arbitrary (bucket reductions are sums / products of group elements)
__global__ void __launch_bounds__(256) bucket_hist_kernel(const int32_t *keys, int64_t n, int64_t nb,
                                                          int32_t *counts) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int32_t k = keys[i];
  if (k >= 0 && k < nb) atomicAdd(&counts[k], 1);
}

__global__ void __launch_bounds__(256) bucket_scatter_kernel(const int32_t *keys, const int32_t *items, int64_t n,
                                                             int64_t nb, const int64_t *offs, int32_t *cursor,
                                                             int32_t *out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int32_t k = keys[i];
  if (k < 0 || k >= nb) return;
  out[offs[k] + atomicAdd(&cursor[k], 1)] = items[i];
}

// slice t of a pass: its bucket b by binary search over the slice offsets
// (one thread per slice: coalesced writes)
__global__ void __launch_bounds__(256) slice_desc_kernel(const int64_t *first, const int64_t *count,
                                                         const int64_t *soff, int sl, int64_t nbk, int64_t total,
                                                         int64_t *st, int32_t *ln) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= total) return;
  int64_t lo = 0, hi = nbk - 1;
  while (lo < hi) {  // last b with soff[b] <= t
    const int64_t mid = (lo + hi + 1) >> 1;
    if (soff[mid] <= t) lo = mid; else hi = mid - 1;
  }
  const int64_t j = t - soff[lo];
  st[t] = first[lo] + j * sl;
  const int64_t rem = count[lo] - j * sl;
  ln[t] = (int32_t)(rem < sl ? rem : sl);
}

inline dim3 blocks(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

}  // namespace

extern "C" {

// temporary storage the device sort needs for n pairs
int dx_bucket_sort_tmp(int64_t n, int end_bit, uint64_t *bytes) {
  size_t tb = 0;
  hipError_t e = rocprim::radix_sort_pairs(nullptr, tb, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                           (const uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)n, 0u,
                                           (unsigned)end_bit);
  *bytes = (uint64_t)tb;
  return e == hipSuccess ? 0 : dx::check_hip(e, "bucket_sort_tmp");
}

int dx_bucket_sort(int on_gpu, void *stream, const int32_t *kin, const int32_t *iin, int32_t *kout, int32_t *iout,
                   int64_t n, int end_bit, void *tmp, uint64_t tmp_bytes) {
  if (n <= 0) return 0;
  if (!on_gpu) {
    const uint32_t mask = end_bit >= 32 ? 0xffffffffu : ((1u << end_bit) - 1u);
    std::vector<int64_t> ord((size_t)n);
    std::iota(ord.begin(), ord.end(), (int64_t)0);
    std::stable_sort(ord.begin(), ord.end(),
                     [&](int64_t a, int64_t b) { return ((uint32_t)kin[a] & mask) < ((uint32_t)kin[b] & mask); });
    for (int64_t i = 0; i < n; i++) {
      kout[i] = kin[ord[i]];
      iout[i] = iin[ord[i]];
    }
    return 0;
  }
  size_t tb = (size_t)tmp_bytes;
  hipError_t e = rocprim::radix_sort_pairs(tmp, tb, (const uint32_t *)kin, (uint32_t *)kout, (const uint32_t *)iin,
                                           (uint32_t *)iout, (size_t)n, 0u, (unsigned)end_bit, (hipStream_t)stream);
  return dx::check_hip(e, "bucket_sort");
}

// first[k] / end[k]: the run of bucket k in the sorted keys (arrays zeroed by the caller)
int dx_bucket_bounds(int on_gpu, void *stream, const int32_t *keys, int64_t n, int64_t nb, int64_t *first,
                     int64_t *end) {
  if (n <= 0) return 0;
  if (!on_gpu) {
    for (int64_t i = 0; i < n; i++) {
      const int32_t k = keys[i];
      if (k < 0 || k >= nb) continue;
      if (i == 0 || keys[i - 1] != k) first[k] = i;
      if (i + 1 == n || keys[i + 1] != k) end[k] = i + 1;
    }
    return 0;
  }
  hipLaunchKernelGGL(bucket_bounds_kernel, blocks(n), dim3(256), 0, (hipStream_t)stream, keys, n, nb, first, end);
  return dx::check_hip(hipGetLastError(), "bucket_bounds");
}

// counts[k] (zeroed int32 [nb]) of the entries with key k < nb
int dx_bucket_hist(int on_gpu, void *stream, const int32_t *keys, int64_t n, int64_t nb, int32_t *counts) {
  if (n <= 0) return 0;
  if (!on_gpu) {
    for (int64_t i = 0; i < n; i++)
      if (keys[i] >= 0 && keys[i] < nb) counts[keys[i]]++;
    return 0;
  }
  hipLaunchKernelGGL(bucket_hist_kernel, blocks(n), dim3(256), 0, (hipStream_t)stream, keys, n, nb, counts);
  return dx::check_hip(hipGetLastError(), "bucket_hist");
}

// out[offs[k] + r] = items of the entries with key k (offs: exclusive prefix
// sums of the counts; cursor zeroed int32 [nb])
int dx_bucket_scatter(int on_gpu, void *stream, const int32_t *keys, const int32_t *items, int64_t n, int64_t nb,
                      const int64_t *offs, int32_t *cursor, int32_t *out) {
  if (n <= 0) return 0;
  if (!on_gpu) {
    for (int64_t i = 0; i < n; i++) {
      const int32_t k = keys[i];
      if (k >= 0 && k < nb) out[offs[k] + cursor[k]++] = items[i];
    }
    return 0;
  }
  hipLaunchKernelGGL(bucket_scatter_kernel, blocks(n), dim3(256), 0, (hipStream_t)stream, keys, items, n, nb, offs,
                     cursor, out);
  return dx::check_hip(hipGetLastError(), "bucket_scatter");
}

// per non-empty bucket b (count[b] entries from first[b]): its slices of <= sl
// entries at soff[b] .. in (st, ln); total = the number of slices
int dx_slice_desc(int on_gpu, void *stream, const int64_t *first, const int64_t *count, const int64_t *soff, int sl,
                  int64_t nbk, int64_t total, int64_t *st, int32_t *ln) {
  if (nbk <= 0 || total <= 0) return 0;
  if (!on_gpu) {
    for (int64_t b = 0; b < nbk; b++) {
      const int64_t ns = (count[b] + sl - 1) / sl;
      for (int64_t j = 0; j < ns; j++) {
        st[soff[b] + j] = first[b] + j * sl;
        ln[soff[b] + j] = (int32_t)std::min<int64_t>(sl, count[b] - j * sl);
      }
    }
    return 0;
  }
  hipLaunchKernelGGL(slice_desc_kernel, blocks(total), dim3(256), 0, (hipStream_t)stream, first, count, soff, sl, nbk,
                     total, st, ln);
  return dx::check_hip(hipGetLastError(), "slice_desc");
}

// per non-empty bucket b (count[b] entries from first[b]): its slices of <= sl
// entries at soff[b] .. in (st, ln)
int dx_slice_plan(int on_gpu, void *stream, const int64_t *first, const int64_t *count, const int64_t *soff, int sl,
                  int64_t nbk, int64_t *st, int32_t *ln) {
  if (nbk <= 0) return 0;
  if (!on_gpu) {
    dx::host_for_each(nbk, [=](int64_t b) {
      const int64_t c = count[b], f = first[b], o = soff[b];
      const int64_t ns = (c + sl - 1) / sl;
      for (int64_t j = 0; j < ns; j++) {
        st[o + j] = f + j * sl;
        ln[o + j] = (int32_t)std::min<int64_t>(sl, c - j * sl);
      }
    });
    return 0;
  }
  hipLaunchKernelGGL(slice_plan_kernel, blocks(nbk), dim3(256), 0, (hipStream_t)stream, first, count, soff, sl, nbk,
                     st, ln);
  return dx::check_hip(hipGetLastError(), "slice_plan");
}

}  // extern "C"
