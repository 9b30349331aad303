// Elementwise epilogue kernels around the SpMM hops (HBM streaming, float4 vectorised).
//   forward : nn.LeakyReLU / nn.ReLU applied after the second hop (HGCNConv act=True,
//             model/graph/HGNN_HD4.py:459-460, model/graph/HGCN.py:171-173) when it cannot be
//             fused into hgd_spmm's store (negative slope).
//   backward: dZ = dY * (ref > 0 ? 1 : slope) — torch's leaky_relu_backward on the saved
//             pre-activation, or on the output when slope >= 0 (same sign).
//   sum_slices: the layer sum of HCCF's encoder, sum(hidden) (model/graph/HCCF.py:188), over
//             the hidden tables stored as slices of one buffer — one pass instead of L adds.
#include <algorithm>

#include "device_util.h"
#include "hgd_internal.h"

namespace hgd {

__device__ __forceinline__ float epi_fwd(float z, int epi, float slope) {
  if (epi == HGD_EPI_LEAKY_RELU) return z > 0.f ? z : z * slope;
  if (epi == HGD_EPI_RELU) return z > 0.f ? z : 0.f;
  return z;
}

__device__ __forceinline__ float epi_bwd(float ref, float dy, int epi, float slope) {
  if (epi == HGD_EPI_LEAKY_RELU) return ref > 0.f ? dy : dy * slope;
  if (epi == HGD_EPI_RELU) return ref > 0.f ? dy : 0.f;
  return dy;
}

__global__ void k_epi_apply(const float* __restrict__ z, int64_t n, int epi, float slope,
                            float* __restrict__ y) {
  const int64_t i4 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) * 4;
  if (i4 + 3 < n) {
    float4 v = *reinterpret_cast<const float4*>(z + i4);
    v.x = epi_fwd(v.x, epi, slope);
    v.y = epi_fwd(v.y, epi, slope);
    v.z = epi_fwd(v.z, epi, slope);
    v.w = epi_fwd(v.w, epi, slope);
    *reinterpret_cast<float4*>(y + i4) = v;
  } else {
    for (int64_t i = i4; i < n; ++i) y[i] = epi_fwd(z[i], epi, slope);
  }
}

__global__ void k_epi_backward(const float* __restrict__ ref, const float* __restrict__ dy,
                               int64_t n, int epi, float slope, float* __restrict__ dz) {
  const int64_t i4 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) * 4;
  if (i4 + 3 < n) {
    const float4 r = *reinterpret_cast<const float4*>(ref + i4);
    float4 g = *reinterpret_cast<const float4*>(dy + i4);
    g.x = epi_bwd(r.x, g.x, epi, slope);
    g.y = epi_bwd(r.y, g.y, epi, slope);
    g.z = epi_bwd(r.z, g.z, epi, slope);
    g.w = epi_bwd(r.w, g.w, epi, slope);
    *reinterpret_cast<float4*>(dz + i4) = g;
  } else {
    for (int64_t i = i4; i < n; ++i) dz[i] = epi_bwd(ref[i], dy[i], epi, slope);
  }
}

// out[i] = ((P_0[i] + P_1[i]) + P_2[i]) + … — Python's sum() order over the slices (its
// leading 0 + P_0 is P_0 exactly), so the result is bit-identical to the chain of adds.
__global__ void k_sum_slices(const float* __restrict__ P, int64_t S, int64_t stride, int64_t n,
                             float* __restrict__ out) {
  const int64_t i4 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) * 4;
  if (i4 + 3 < n) {
    float4 acc = *reinterpret_cast<const float4*>(P + i4);
    for (int64_t s = 1; s < S; ++s) {
      const float4 v = *reinterpret_cast<const float4*>(P + s * stride + i4);
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    *reinterpret_cast<float4*>(out + i4) = acc;
  } else {
    for (int64_t i = i4; i < n; ++i) {
      float acc = P[i];
      for (int64_t s = 1; s < S; ++s) acc += P[s * stride + i];
      out[i] = acc;
    }
  }
}

// out = ((a_0 + a_1) + a_2) + … over up to kMaxSumArrays separate arrays (one pass: n + 1 array
// streams instead of the 3·(n − 1) of a chain of binary adds)
constexpr int kMaxSumArrays = 8;
struct SumArrays {
  const float* a[kMaxSumArrays];
  int32_t n;
};

__global__ void k_sum_arrays(SumArrays A, int64_t count, float* out) {  // out may alias a[0]
  const int64_t i4 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) * 4;
  if (i4 + 3 < count) {
    float4 acc = *reinterpret_cast<const float4*>(A.a[0] + i4);
    for (int s = 1; s < A.n; ++s) {
      const float4 v = *reinterpret_cast<const float4*>(A.a[s] + i4);
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    *reinterpret_cast<float4*>(out + i4) = acc;
  } else {
    for (int64_t i = i4; i < count; ++i) {
      float acc = A.a[0][i];
      for (int s = 1; s < A.n; ++s) acc += A.a[s][i];
      out[i] = acc;
    }
  }
}

// nn.Dropout on the device RNG of dropout_keep4 (device_util.h): y[i] = keep(i) ? x[i]·scale : 0,
// one draw per float4 (its four elements are one keep group). The same call on the upstream
// gradient with the same seed is the backward (no stored mask).
__global__ void k_dropout(const float* __restrict__ x, int64_t n, const uint64_t* __restrict__ seed_p,
                          float keep, float scale, float* __restrict__ y) {
  const uint64_t seed = *seed_p;
  const uint32_t thr = dropout_threshold(keep);
  const int64_t i4 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) * 4;
  if (i4 + 3 < n) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + i4);
    *reinterpret_cast<f32x4*>(y + i4) =
        dropout_apply4(v, seed, static_cast<uint32_t>(i4 >> 2), thr, scale);
  } else {
    for (int64_t i = i4; i < n; ++i)
      y[i] = dropout_keep(seed, static_cast<uint32_t>(i), thr) ? x[i] * scale : 0.f;
  }
}

// The backward of L dropouts of one tensor (torch's native_dropout_backward per call,
// g_k = ((float)mask_k · dy_k) · scale, then autograd's accumulation of the L gradients as they
// arrive, the last call's first): out = ((g_{L-1} + g_{L-2}) + …) + g_0, one pass. Up to
// kMaxMaskedSum calls per tensor and kMaxMaskedJobs tensors per launch (blockIdx.y). No
// contraction: torch rounds the product and the sums separately.
constexpr int kMaxMaskedSum = 8;
constexpr int kMaxMaskedJobs = 4;
struct MaskedSumJob {
  const float* dy[kMaxMaskedSum];
  const uint8_t* mask[kMaxMaskedSum];
  float* out;
  int64_t n;
  int32_t count;
  float scale;
};
struct MaskedSumJobs {
  MaskedSumJob j[kMaxMaskedJobs];
};

#pragma clang fp contract(off)
__global__ void k_masked_scale_sum(MaskedSumJobs J) {
  const MaskedSumJob& b = J.j[blockIdx.y];
  const int64_t i4 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) * 4;
  if (i4 >= b.n) return;
  const int L = b.count;
  if (i4 + 3 < b.n) {
    float acc[4];
    for (int k = L - 1; k >= 0; --k) {
      const f32x4 d = *reinterpret_cast<const f32x4*>(b.dy[k] + i4);
      const uint32_t m = *reinterpret_cast<const uint32_t*>(b.mask[k] + i4);
      float g[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float mf = ((m >> (8 * t)) & 0xffu) ? 1.f : 0.f;
        g[t] = (mf * d[t]) * b.scale;
        acc[t] = k == L - 1 ? g[t] : acc[t] + g[t];
      }
    }
    f32x4 o;
#pragma unroll
    for (int t = 0; t < 4; ++t) o[t] = acc[t];
    *reinterpret_cast<f32x4*>(b.out + i4) = o;
  } else {
    for (int64_t i = i4; i < b.n; ++i) {
      float acc = 0.f;
      for (int k = L - 1; k >= 0; --k) {
        const float g = ((b.mask[k][i] ? 1.f : 0.f) * b.dy[k][i]) * b.scale;
        acc = k == L - 1 ? g : acc + g;
      }
      b.out[i] = acc;
    }
  }
}
#pragma clang fp contract(on)

inline bool aligned16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }

}  // namespace hgd

using namespace hgd;

extern "C" hgd_status hgd_epilogue_apply(const float* z, int64_t n, int32_t epilogue, float slope,
                                         float* y, void* stream) {
  clear_error();
  HGD_REQUIRE(n >= 0, "hgd_epilogue_apply: n < 0");
  if (n == 0) return HGD_OK;
  HGD_REQUIRE(z && y && aligned16(z) && aligned16(y), "hgd_epilogue_apply: null/unaligned");
  hipLaunchKernelGGL(k_epi_apply, dim3(grid_for((n + 3) / 4)), dim3(kBlock), 0,
                     as_stream(stream), z, n, epilogue, slope, y);
  return check_launch("hgd_epilogue_apply");
}

extern "C" hgd_status hgd_epilogue_backward(const float* ref, const float* dy, int64_t n,
                                            int32_t epilogue, float slope, float* dz,
                                            void* stream) {
  clear_error();
  HGD_REQUIRE(n >= 0, "hgd_epilogue_backward: n < 0");
  if (n == 0) return HGD_OK;
  HGD_REQUIRE(ref && dy && dz && aligned16(ref) && aligned16(dy) && aligned16(dz),
              "hgd_epilogue_backward: null/unaligned");
  hipLaunchKernelGGL(k_epi_backward, dim3(grid_for((n + 3) / 4)), dim3(kBlock), 0,
                     as_stream(stream), ref, dy, n, epilogue, slope, dz);
  return check_launch("hgd_epilogue_backward");
}

extern "C" hgd_status hgd_sum_slices(const float* P, int64_t n_slices, int64_t slice_stride,
                                     int64_t n, float* out, void* stream) {
  clear_error();
  HGD_REQUIRE(n >= 0 && n_slices >= 1 && slice_stride >= n, "hgd_sum_slices: bad sizes");
  if (n == 0) return HGD_OK;
  HGD_REQUIRE(P && out && aligned16(P) && aligned16(out) && slice_stride % 4 == 0,
              "hgd_sum_slices: null/unaligned (16-byte slices needed)");
  hipLaunchKernelGGL(k_sum_slices, dim3(grid_for((n + 3) / 4)), dim3(kBlock), 0,
                     as_stream(stream), P, n_slices, slice_stride, n, out);
  return check_launch("hgd_sum_slices");
}

extern "C" hgd_status hgd_sum_arrays(const float* const* arrays, int32_t n_arrays,
                                     int64_t count, float* out, void* stream) {
  clear_error();
  HGD_REQUIRE(arrays && n_arrays >= 1 && n_arrays <= kMaxSumArrays && count >= 0,
              "hgd_sum_arrays: 1..%d arrays, count >= 0", kMaxSumArrays);
  if (count == 0) return HGD_OK;
  SumArrays A{};
  A.n = n_arrays;
  for (int s = 0; s < n_arrays; ++s) {
    HGD_REQUIRE(arrays[s] && aligned16(arrays[s]), "hgd_sum_arrays: array %d null/unaligned", s);
    A.a[s] = arrays[s];
  }
  HGD_REQUIRE(out && aligned16(out), "hgd_sum_arrays: out null/unaligned");
  hipLaunchKernelGGL(k_sum_arrays, dim3(grid_for((count + 3) / 4)), dim3(kBlock), 0,
                     as_stream(stream), A, count, out);
  return check_launch("hgd_sum_arrays");
}

extern "C" hgd_status hgd_dropout_apply(const float* x, int64_t n, const uint64_t* seed,
                                        float keep, float scale, float* y, void* stream) {
  clear_error();
  HGD_REQUIRE(n >= 0, "hgd_dropout_apply: n < 0");
  HGD_REQUIRE(keep > 0.f && keep <= 1.f, "hgd_dropout_apply: keep must be in (0, 1]");
  HGD_REQUIRE(n <= 0xffffffffLL, "hgd_dropout_apply: n must be < 2^32 (32-bit element counter)");
  if (n == 0) return HGD_OK;
  HGD_REQUIRE(x && y && seed && aligned16(x) && aligned16(y), "hgd_dropout_apply: null/unaligned");
  hipLaunchKernelGGL(k_dropout, dim3(grid_for((n + 3) / 4)), dim3(kBlock), 0, as_stream(stream),
                     x, n, seed, keep, scale, y);
  return check_launch("hgd_dropout_apply");
}

extern "C" hgd_status hgd_masked_scale_sum(const hgd_masked_sum* jobs, int32_t n_jobs,
                                           void* stream) {
  clear_error();
  HGD_REQUIRE(jobs && n_jobs >= 1 && n_jobs <= kMaxMaskedJobs,
              "hgd_masked_scale_sum: 1..%d jobs", kMaxMaskedJobs);
  MaskedSumJobs J{};
  int64_t n_max = 0;
  for (int q = 0; q < n_jobs; ++q) {
    const hgd_masked_sum& d = jobs[q];
    HGD_REQUIRE(d.count >= 1 && d.count <= kMaxMaskedSum && d.n >= 0,
                "hgd_masked_scale_sum: job %d: 1..%d gradients, n >= 0", q, kMaxMaskedSum);
    HGD_REQUIRE(d.out && aligned16(d.out), "hgd_masked_scale_sum: job %d: out null/unaligned", q);
    MaskedSumJob& b = J.j[q];
    for (int k = 0; k < d.count; ++k) {
      HGD_REQUIRE(d.dy[k] && d.mask[k] && aligned16(d.dy[k]) &&
                      reinterpret_cast<uintptr_t>(d.mask[k]) % 4 == 0,
                  "hgd_masked_scale_sum: job %d: dy / mask %d null or unaligned", q, k);
      b.dy[k] = d.dy[k];
      b.mask[k] = d.mask[k];
    }
    b.out = d.out;
    b.n = d.n;
    b.count = d.count;
    b.scale = d.scale;
    n_max = std::max<int64_t>(n_max, d.n);
  }
  if (n_max == 0) return HGD_OK;
  hipLaunchKernelGGL(k_masked_scale_sum, dim3(grid_for((n_max + 3) / 4), n_jobs), dim3(kBlock), 0,
                     as_stream(stream), J);
  return check_launch("hgd_masked_scale_sum");
}
