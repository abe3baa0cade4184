// Bucket plans of the Pippenger MSMs / multi-exponentiations (G1, G2, GT):
// the (group, window, digit) keys of every scalar entry are sorted with their
// entry index (torch's onesweep radix sort), then
//
//  * dx_bucket_bounds: first entry and end of every bucket's run in the sorted
//    keys (run boundaries only: coalesced reads, one write per boundary).
//  * dx_lane_slices: device-resident plans -- every bucket owns a FIXED number
//    of lanes (chosen from the plan's shape: the expected entries per digit
//    of its window), and lane j of bucket b takes the j-th of its lanes'
//    equal shares of the bucket's actual run.  Nothing about the plan goes
//    through the host, so the reduction passes are queued at once (no host
//    sync on the counts); skewed buckets only get longer slices.
//  * dx_slice_desc: host-planned passes (the segment-grouped attribution
//    pass): one thread per slice (binary search of its bucket) writes the pass
//    descriptors (start, length), coalesced.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

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

// lane t of bucket b = lane_bucket[t] (lane_j[t] of its lanes[b]): an equal
// share of the bucket's run [first[b], end[b]) -- one lane per slice of the
// reduction's first pass
__global__ void __launch_bounds__(256) lane_slices_kernel(const int64_t *first, const int64_t *end,
                                                          const int32_t *lane_bucket, const int32_t *lane_j,
                                                          const int32_t *lanes, int64_t n_lanes, int64_t *st,
                                                          int32_t *ln) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n_lanes) return;
  const int32_t b = lane_bucket[t];
  const int64_t f = first[b], cnt = end[b] - f, L = lanes[b];
  const int64_t per = (cnt + L - 1) / L, a = (int64_t)lane_j[t] * per;
  st[t] = f + a;
  ln[t] = (int32_t)(cnt > a ? (cnt - a < per ? cnt - a : per) : 0);
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

// lane slices of a device-resident plan (see lane_slices_kernel)
int dx_lane_slices(int on_gpu, void *stream, const int64_t *first, const int64_t *end, const int32_t *lane_bucket,
                   const int32_t *lane_j, const int32_t *lanes, int64_t n_lanes, int64_t *st, int32_t *ln) {
  if (n_lanes <= 0) return 0;
  if (!on_gpu) {
    for (int64_t t = 0; t < n_lanes; t++) {
      const int32_t b = lane_bucket[t];
      const int64_t f = first[b], cnt = end[b] - f, L = lanes[b];
      const int64_t per = (cnt + L - 1) / L, a = (int64_t)lane_j[t] * per;
      st[t] = f + a;
      ln[t] = (int32_t)(cnt > a ? std::min<int64_t>(cnt - a, per) : 0);
    }
    return 0;
  }
  hipLaunchKernelGGL(lane_slices_kernel, blocks(n_lanes), dim3(256), 0, (hipStream_t)stream, first, end, lane_bucket,
                     lane_j, lanes, n_lanes, st, ln);
  return dx::check_hip(hipGetLastError(), "lane_slices");
}

}  // extern "C"
