// Shared helpers for the batched-op translation units.
#pragma once
#include <cstring>
#include "../bn254/pairing.h"
#include "exec.h"

using namespace dx;

namespace dxk {

template <class T>
DX_HD const T &at(const uint32_t *base, int64_t i) {
  return reinterpret_cast<const T *>(base)[i];
}
template <class T>
DX_HD T &at(uint32_t *base, int64_t i) {
  return reinterpret_cast<T *>(base)[i];
}

DX_HD void signed_to_scalar(int64_t m, uint32_t *k, bool &negate) {
  negate = m < 0;
  uint64_t a = negate ? (uint64_t)(-(m + 1)) + 1ull : (uint64_t)m;
  k[0] = (uint32_t)a;
  k[1] = (uint32_t)(a >> 32);
  for (int i = 2; i < 8; i++) k[i] = 0;
}

DX_HD bool cas64(uint64_t *addr, uint64_t expected, uint64_t desired, uint64_t &old) {
#ifdef __HIP_DEVICE_COMPILE__
  old = atomicCAS((unsigned long long *)addr, (unsigned long long)expected, (unsigned long long)desired);
  return old == expected;
#else
  uint64_t e = expected;
  bool ok = __atomic_compare_exchange_n(addr, &e, desired, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);
  old = e;
  return ok;
#endif
}

DX_HD uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// key of an affine point for the BSGS table: 63 bits of canonical-free x limbs
// (Montgomery x is a bijection of x, so hashing it directly is fine); 0 = empty.
DX_HD uint64_t point_key(const G1A &a) {
  uint64_t k = ((uint64_t)a.x.v[1] << 32) | a.x.v[0];
  k ^= ((uint64_t)a.x.v[3] << 32 | a.x.v[2]) * 0x9E3779B97F4A7C15ull;
  k |= 1ull;  // never 0
  return k;
}

}  // namespace dxk


using namespace dxk;
