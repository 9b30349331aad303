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

// SplitMix64 finaliser (the counter-based RNGs of the device drop-edge and dropout draws).
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// 32-bit integer finaliser ("lowbias32": two multiplies, three xor-shifts).
__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// Dropout keep-bit of element i (< 2^32) of a draw (nn.Dropout(p): keep with probability
// keep = 1 - p): h = lowbias32(lowbias32(i + lo32(seed)) ^ hi32(seed)), u = (h >> 8)·2^-24,
// kept iff floor(u + keep) != 0 — 32-bit arithmetic only, so it costs a few VALU slots beside
// the MFMAs of the Linear it rides in (oracle: hgd_oracle.dropout_keep_mask).
__device__ __forceinline__ bool dropout_keep(uint64_t seed, uint32_t i, float keep) {
  const uint32_t h = lowbias32(lowbias32(i + static_cast<uint32_t>(seed)) ^
                               static_cast<uint32_t>(seed >> 32));
  const float u = static_cast<float>(h >> 8) * (1.0f / 16777216.0f);
  return floorf(u + keep) != 0.f;
}

inline int next_pow2(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}

}  // namespace hgd
