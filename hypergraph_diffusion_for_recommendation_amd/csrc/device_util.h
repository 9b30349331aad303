// Device helpers shared by the libhgd kernels (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>

namespace hgd {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Sum of v over the G lanes of this lane group (xor butterfly; every lane gets the total).
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int m = G / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, G);
  return v;
}

// v_mfma_f32_16x16x4_f32: exact f32 products and sums at the f32 vector rate. Lane l supplies
// A[l & 15][l >> 4] and B[l >> 4][l & 15]; C/D register r of lane l is row 4(l >> 4) + r,
// column l & 15.
__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// VEC contiguous floats (one 16-byte access when VEC == 4; NT = non-temporal).
template <int VEC, bool NT = false>
__device__ __forceinline__ void load_vec(const float* p, float (&v)[VEC]) {
  if constexpr (VEC == 4) {
    f32x4 t;
    if constexpr (NT)
      t = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    else
      t = *reinterpret_cast<const f32x4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else {
#pragma unroll
    for (int i = 0; i < VEC; ++i) v[i] = p[i];
  }
}

template <int VEC, bool NT = false>
__device__ __forceinline__ void store_vec(float* p, const float (&v)[VEC]) {
  if constexpr (VEC == 4) {
    const f32x4 t = {v[0], v[1], v[2], v[3]};
    if constexpr (NT)
      __builtin_nontemporal_store(t, reinterpret_cast<f32x4*>(p));
    else
      *reinterpret_cast<f32x4*>(p) = t;
  } else {
#pragma unroll
    for (int i = 0; i < VEC; ++i) p[i] = v[i];
  }
}

inline int next_pow2(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}

}  // namespace hgd
