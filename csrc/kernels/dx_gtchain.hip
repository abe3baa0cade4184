// Latency-hidden GT product chains (the bucket accumulation of the verifier's
// multi-exponentiations, K8; lib/range/range_proof.go:540-546 multiplies the
// a_ij into GT products one by one).
//
//   out[s] = prod_{k < len[s]} src[idx ? idx[start[s] + k] : start[s] + k]
//
// Each step multiplies a 384-byte Fp12 gathered from an arbitrary row of a
// multi-GB array: on gfx950 the product (18 Fp2 multiplications) is short
// next to the latency of that gather, and the previous build
// (dx_gt_slice_prod: out-of-line tower functions, 2 waves per SIMD) spilled
// ~1.8 KiB of Fp12 temporaries per lane and issued VALU a third of its
// lifetime.  Here the whole chain is force-inlined into one kernel that owns
// the register file of a SIMD lane (1 wave per SIMD: 512 registers, no
// scratch), and the gather of element k+1 -- and the index of element k+2
// -- are issued BEFORE the product with element k, so the HBM latency
// overlaps the arithmetic instead of stalling it.
#define DX_NI __host__ __device__ __forceinline__
#include "common.h"

using namespace dxk;

namespace {
constexpr int kGW = 64;

DX_HD void gt_chain_one(const uint32_t *src, const int64_t *idx, const int64_t *start, const int32_t *len,
                        uint32_t *out, int64_t s) {
  const int64_t b = start[s];
  const int n = len[s];
  Fp12 acc = Fp12::one();
  if (n > 0) {
    int64_t i_next = idx ? idx[b] : b;
    int64_t i_after = (n > 1) ? (idx ? idx[b + 1] : b + 1) : 0;
    Fp12 nxt = at<Fp12>(src, i_next);
    for (int k = 0; k < n; k++) {
      const Fp12 cur = nxt;
      if (k + 1 < n) {
        nxt = at<Fp12>(src, i_after);  // gather of k+1 in flight during the product with k
        if (k + 2 < n) i_after = idx ? idx[b + k + 2] : b + k + 2;
      }
      acc = mul(acc, cur);
    }
  }
  at<Fp12>(out, s) = acc;
}

__global__ void __launch_bounds__(kGW) __attribute__((amdgpu_waves_per_eu(1, 1)))
gt_chain_kernel(const uint32_t *src, const int64_t *idx, const int64_t *start, const int32_t *len, uint32_t *out,
                int64_t n) {
  const int64_t s = (int64_t)blockIdx.x * kGW + threadIdx.x;
  if (s < n) gt_chain_one(src, idx, start, len, out, s);
}
}  // namespace

extern "C" int dx_gt_chain(int on_gpu, void *stream, const uint32_t *src, const int64_t *idx, const int64_t *start,
                           const int32_t *len, uint32_t *out, int64_t n_slices) {
  if (n_slices <= 0) return 0;
  if (!on_gpu) {
    host_for_each(n_slices, [=](int64_t s) { gt_chain_one(src, idx, start, len, out, s); });
    return 0;
  }
  hipLaunchKernelGGL(gt_chain_kernel, dim3((unsigned)((n_slices + kGW - 1) / kGW)), dim3(kGW), 0,
                     (hipStream_t)stream, src, idx, start, len, out, n_slices);
  return check_hip(hipGetLastError(), "gt_chain");
}
