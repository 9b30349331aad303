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

// Dropout keep-bits (nn.Dropout(p): keep with probability keep = 1 - p), counter-based and drawn
// for four consecutive elements at once — elements 4c .. 4c + 3 of a draw (c < 2^30) take the
// four 16-bit halves of h1 = lowbias32(lowbias32(c + lo32(seed)) ^ hi32(seed)) and
// h2 = lowbias32(h1 ^ 0x9E3779B9) (low half first); an element is kept iff its half is below
// thr = dropout_threshold(keep) = ⌊keep·2^16 + 1/2⌋ (f32 arithmetic). Three 32-bit finalisers per
// four elements (the per-element form took two per element, up to 60 % of a d = 128 Linear
// with the dropout in its store); bit s of the result is element 4c + s (oracle:
// hgd_oracle.dropout_keep_mask).
__device__ __forceinline__ uint32_t dropout_threshold(float keep) {
  return static_cast<uint32_t>(keep * 65536.0f + 0.5f);
}

__device__ __forceinline__ uint32_t dropout_keep4(uint64_t seed, uint32_t c, uint32_t thr) {
  const uint32_t h1 = lowbias32(lowbias32(c + static_cast<uint32_t>(seed)) ^
                                static_cast<uint32_t>(seed >> 32));
  const uint32_t h2 = lowbias32(h1 ^ 0x9E3779B9u);
  return static_cast<uint32_t>((h1 & 0xffffu) < thr) |
         (static_cast<uint32_t>((h1 >> 16) < thr) << 1) |
         (static_cast<uint32_t>((h2 & 0xffffu) < thr) << 2) |
         (static_cast<uint32_t>((h2 >> 16) < thr) << 3);
}

// Keep-bit of one element i (< 2^32) of the same draw.
__device__ __forceinline__ bool dropout_keep(uint64_t seed, uint32_t i, uint32_t thr) {
  return (dropout_keep4(seed, i >> 2, thr) >> (i & 3u)) & 1u;
}

// v ⊙ keep-bits × scale for the four elements 4c .. 4c + 3 held in v
__device__ __forceinline__ f32x4 dropout_apply4(f32x4 v, uint64_t seed, uint32_t c, uint32_t thr,
                                                float scale) {
  const uint32_t k = dropout_keep4(seed, c, thr);
  return f32x4{(k & 1u) ? v.x * scale : 0.f, (k & 2u) ? v.y * scale : 0.f,
               (k & 4u) ? v.z * scale : 0.f, (k & 8u) ? v.w * scale : 0.f};
}

inline int next_pow2(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}

}  // namespace hgd
