// Bucket plans of the Pippenger MSMs / multi-exponentiations (G1, G2, GT):
// the entries (entry index by (group, window, digit) key) are grouped by
// bucket with a counting sort (dx_bucket_sort: histogram, scan, scatter), then
//
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

// Counting sort of the plan's entries by bucket key (replaces a device radix
// sort of the keys: one histogram pass and one scatter pass instead of four
// onesweep passes, and no library sort inside the verifier's HIP graphs).
// Entries of one bucket land in arbitrary order -- every consumer sums its
// bucket (exact group arithmetic, order-free).  Zero-digit sentinel keys
// (outside [0, nb)) are dropped.
__global__ void __launch_bounds__(256) key_hist_kernel(const int32_t *keys, int64_t n, int64_t nb, uint32_t *count) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const int32_t k = keys[i];
    if (k >= 0 && k < nb) atomicAdd(&count[k], 1u);
  }
}

constexpr int kScanTile = 1024;  // 256 threads x 4 buckets

// exclusive scan of each 1024-bucket tile (int64), the tile totals to `tot`
__global__ void __launch_bounds__(256) scan_tile_kernel(const uint32_t *count, int64_t nb, int64_t *first,
                                                        int64_t *tot) {
  __shared__ int64_t s[256];
  const int t = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * kScanTile + 4 * t;
  int64_t v[4], sum = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    v[k] = base + k < nb ? (int64_t)count[base + k] : 0;
    sum += v[k];
  }
  s[t] = sum;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    const int64_t x = t >= off ? s[t - off] : 0;
    __syncthreads();
    s[t] += x;
    __syncthreads();
  }
  int64_t e = s[t] - sum;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (base + k < nb) first[base + k] = e;
    e += v[k];
  }
  if (t == 255) tot[blockIdx.x] = s[255];
}

// exclusive scan of the tile totals in place: one workgroup, 1024 at a time
__global__ void __launch_bounds__(1024) scan_tot_kernel(int64_t *tot, int64_t n_tiles) {
  __shared__ int64_t s[1024];
  __shared__ int64_t carry;
  const int t = threadIdx.x;
  if (t == 0) carry = 0;
  __syncthreads();
  for (int64_t b0 = 0; b0 < n_tiles; b0 += 1024) {
    const int64_t v = b0 + t < n_tiles ? tot[b0 + t] : 0;
    s[t] = v;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const int64_t x = t >= off ? s[t - off] : 0;
      __syncthreads();
      s[t] += x;
      __syncthreads();
    }
    if (b0 + t < n_tiles) tot[b0 + t] = carry + s[t] - v;
    __syncthreads();
    if (t == 1023) carry += s[1023];
    __syncthreads();
  }
}

// first += its tile's offset; end = first + count; the scatter cursors start at first
__global__ void __launch_bounds__(256) scan_add_kernel(const uint32_t *count, int64_t nb, const int64_t *tot,
                                                       int64_t *first, int64_t *end, uint32_t *cursor) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nb) return;
  const int64_t f = first[i] + tot[i / kScanTile];
  first[i] = f;
  end[i] = f + count[i];
  cursor[i] = (uint32_t)f;
}

__global__ void __launch_bounds__(256) key_scatter_kernel(const int32_t *keys, const int32_t *items, int64_t n,
                                                          int64_t nb, uint32_t *cursor, int32_t *out) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const int32_t k = keys[i];
    if (k >= 0 && k < nb) out[atomicAdd(&cursor[k], 1u)] = items[i];
  }
}

inline dim3 blocks(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }
inline dim3 stride_blocks(int64_t n) {  // grid-stride passes: <= 8 workgroups per CU of 256 CUs
  const int64_t b = (n + 255) / 256;
  return dim3((unsigned)(b < 2048 ? (b > 0 ? b : 1) : 2048));
}

}  // namespace

extern "C" {

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

// Bucket runs of n (key, item) entries: out = the items grouped by key (keys
// in [0, nb); others dropped), first / end = every bucket's run in out.
// Scratch: count, cursor [nb] uint32 and tot [ceil(nb / 1024)] int64.
int dx_bucket_sort(int on_gpu, void *stream, const int32_t *keys, const int32_t *items, int64_t n, int64_t nb,
                   uint32_t *count, uint32_t *cursor, int64_t *tot, int64_t *first, int64_t *end, int32_t *out) {
  if (nb <= 0) return 0;
  if (n >= (int64_t)1 << 32) return -2;
  const int64_t n_tiles = (nb + kScanTile - 1) / kScanTile;
  if (!on_gpu) {
    std::fill(count, count + nb, 0u);
    for (int64_t i = 0; i < n; i++)
      if (keys[i] >= 0 && keys[i] < nb) count[keys[i]]++;
    int64_t acc = 0;
    for (int64_t b = 0; b < nb; b++) {
      first[b] = acc;
      acc += count[b];
      end[b] = acc;
      cursor[b] = (uint32_t)first[b];
    }
    for (int64_t i = 0; i < n; i++)
      if (keys[i] >= 0 && keys[i] < nb) out[cursor[keys[i]]++] = items[i];
    return 0;
  }
  hipStream_t s = (hipStream_t)stream;
  if (dx::check_hip(hipMemsetAsync(count, 0, (size_t)nb * 4, s), "bucket_sort memset")) return -1;
  if (n > 0) hipLaunchKernelGGL(key_hist_kernel, stride_blocks(n), dim3(256), 0, s, keys, n, nb, count);
  hipLaunchKernelGGL(scan_tile_kernel, dim3((unsigned)n_tiles), dim3(256), 0, s, count, nb, first, tot);
  hipLaunchKernelGGL(scan_tot_kernel, dim3(1), dim3(1024), 0, s, tot, n_tiles);
  hipLaunchKernelGGL(scan_add_kernel, blocks(nb), dim3(256), 0, s, count, nb, tot, first, end, cursor);
  if (n > 0) hipLaunchKernelGGL(key_scatter_kernel, stride_blocks(n), dim3(256), 0, s, keys, items, n, nb, cursor, out);
  return dx::check_hip(hipGetLastError(), "bucket_sort");
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
