// The reference's optimizer step as ONE kernel that a HIP graph can hold: torch.optim.Adam(lr=…)
// (model/graph/HCCF.py:33) — the non-capturable multi-tensor form torch runs on the device, whose
// per-step scalars are Python doubles computed on the host (bias corrections of the step count):
//
//   m ← lerp(m, g, 1 − β1)                    torch._foreach_lerp_ (weight < 0.5: m + w·(g − m))
//   v ← v·β2 ; v ← v + (1 − β2)·(g·g)         torch._foreach_mul_ / _foreach_addcmul_
//   d ← sqrt(v) / sqrt(1 − β2^t) + eps        torch._foreach_sqrt / _foreach_div_ / _foreach_add_
//   p ← p + (−lr / (1 − β1^t))·(m / d)        torch._foreach_addcdiv_
//
// Every scalar enters those kernels rounded to float (their opmath), so here they are read from a
// device table of such rows — one per step, the host fills it for many steps ahead and the launch
// advances a device row index after use, so a replayed graph needs no host work per step — and
// each op's rounding is reproduced in its order. Whether torch's build contracted a multiply-add into
// an fma, and which square root / division it emits, is not visible from Python: `variant` picks
// each (bit 0: lerp fused, bit 1: addcmul fused, bit 2: addcdiv fused, bit 3: fast sqrt, bit 4:
// fast division), and tests/test_gpu_adam.py finds the one that is bitwise torch's on this image.
#include "device_util.h"
#include "hgd_internal.h"

namespace hgd {
namespace {

constexpr int kMaxAdamTensors = 16;
constexpr int kAdamChunk = 4096;  // elements per workgroup: 256 threads × 4 float4s

struct AdamList {
  float* p[kMaxAdamTensors];
  const float* g[kMaxAdamTensors];
  float* m[kMaxAdamTensors];
  float* v[kMaxAdamTensors];
  int64_t n[kMaxAdamTensors];
  int32_t block0[kMaxAdamTensors + 1];  // first workgroup of each tensor
  int32_t vec[kMaxAdamTensors];         // 1: the four arrays are 16-byte aligned
  int32_t count;
};

// No contraction anywhere here: a multiply-add is an fma only where `fused` asks for one.
__device__ __forceinline__ float mul_add(float a, float b, float c, bool fused) {
#pragma clang fp contract(off)
  return fused ? __builtin_fmaf(a, b, c) : a * b + c;
}

__device__ __forceinline__ float sqrt_of(float x, bool fast) {
  return fast ? __builtin_amdgcn_sqrtf(x) : __builtin_sqrtf(x);  // the latter correctly rounded
}

__device__ __forceinline__ float div_of(float a, float b, bool fast) {
#pragma clang fp contract(off)
  return fast ? a * __builtin_amdgcn_rcpf(b) : a / b;  // the latter correctly rounded
}

// one element: torch's op order (see the file header), scalars s[0..5]
__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v,
                                         const float* s, int32_t variant) {
#pragma clang fp contract(off)
  const bool f_lerp = variant & 1, f_cmul = variant & 2, f_cdiv = variant & 4;
  const bool fast_sqrt = variant & 8, fast_div = variant & 16;
  // lerp(m, g, w), w = 1 − β1 < 0.5 (ATen Lerp.h: self + weight·(end − self))
  m = mul_add(s[0], g - m, m, f_lerp);
  // v·β2, then addcmul as torch's foreach pointwise functor: v + value·(g·g)
  v = v * s[1];
  v = mul_add(s[2], g * g, v, f_cmul);
  float d = sqrt_of(v, fast_sqrt);
  d = div_of(d, s[3], fast_div);
  d = d + s[4];
  // addcdiv: p + value·(m / d)
  p = mul_add(s[5], div_of(m, d, fast_div), p, f_cdiv);
}

// Workgroup b works on chunk (b − block0[t]) of tensor t: float4 loads and stores when the
// tensor's arrays are aligned, element-wise otherwise (and for the tail).
__global__ __launch_bounds__(256) void k_adam(AdamList L, const float* __restrict__ table,
                                              const int32_t* __restrict__ row,
                                              int32_t variant) {
  const int b = static_cast<int>(blockIdx.x);
  int t = 0;
#pragma unroll 1
  while (t + 1 < L.count && b >= L.block0[t + 1]) ++t;
  const int64_t n = L.n[t];
  const int64_t base = static_cast<int64_t>(b - L.block0[t]) * kAdamChunk;
  const int64_t r = row ? *row : 0;
  const float* s = table + (r * L.count + t) * 6;
  float sc[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) sc[k] = s[k];
  float* P = L.p[t];
  const float* G = L.g[t];
  float* M = L.m[t];
  float* V = L.v[t];
  if (L.vec[t]) {
#pragma unroll
    for (int k = 0; k < kAdamChunk / 1024; ++k) {
      const int64_t e = base + 4 * (threadIdx.x + 256 * k);
      if (e + 4 <= n) {
        f32x4 p4 = *reinterpret_cast<const f32x4*>(P + e);
        const f32x4 g4 = *reinterpret_cast<const f32x4*>(G + e);
        f32x4 m4 = *reinterpret_cast<const f32x4*>(M + e);
        f32x4 v4 = *reinterpret_cast<const f32x4*>(V + e);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float pp = p4[c], mm = m4[c], vv = v4[c];
          adam_one(pp, g4[c], mm, vv, sc, variant);
          p4[c] = pp;
          m4[c] = mm;
          v4[c] = vv;
        }
        *reinterpret_cast<f32x4*>(P + e) = p4;
        *reinterpret_cast<f32x4*>(M + e) = m4;
        *reinterpret_cast<f32x4*>(V + e) = v4;
      } else {
        for (int64_t x = e; x < n && x < e + 4; ++x) adam_one(P[x], G[x], M[x], V[x], sc, variant);
      }
    }
  } else {
    for (int64_t x = base + threadIdx.x; x < n && x < base + kAdamChunk; x += 256)
      adam_one(P[x], G[x], M[x], V[x], sc, variant);
  }
}

// The next replay reads the next row of the step table (after every workgroup has read this one).
__global__ void k_adam_advance(int32_t* row) { *row += 1; }

}  // namespace
}  // namespace hgd

extern "C" hgd_status hgd_adam_step(const hgd_adam_tensor* tensors, int32_t count,
                                    const float* scalars, int32_t* step_row, int32_t variant,
                                    void* stream) {
  hgd::clear_error();
  HGD_REQUIRE(tensors && count >= 1 && count <= hgd::kMaxAdamTensors,
              "hgd_adam_step: 1 to %d tensors", hgd::kMaxAdamTensors);
  HGD_REQUIRE(scalars, "hgd_adam_step: null scalars");
  HGD_REQUIRE(variant >= 0 && variant < 32, "hgd_adam_step: variant in [0, 32)");
  hgd::AdamList L{};
  L.count = count;
  int64_t blocks = 0;
  for (int t = 0; t < count; ++t) {
    const hgd_adam_tensor& x = tensors[t];
    HGD_REQUIRE(x.n >= 0, "hgd_adam_step: tensor %d has a negative size", t);
    HGD_REQUIRE(x.n == 0 || (x.param && x.grad && x.exp_avg && x.exp_avg_sq),
                "hgd_adam_step: tensor %d has a null pointer", t);
    L.p[t] = x.param;
    L.g[t] = x.grad;
    L.m[t] = x.exp_avg;
    L.v[t] = x.exp_avg_sq;
    L.n[t] = x.n;
    auto al = [](const void* q) { return reinterpret_cast<uintptr_t>(q) % 16 == 0; };
    L.vec[t] = al(x.param) && al(x.grad) && al(x.exp_avg) && al(x.exp_avg_sq) ? 1 : 0;
    L.block0[t] = static_cast<int32_t>(blocks);
    blocks += (x.n + hgd::kAdamChunk - 1) / hgd::kAdamChunk;
    HGD_REQUIRE(blocks < 0x7fffffff, "hgd_adam_step: too many elements");
  }
  L.block0[count] = static_cast<int32_t>(blocks);
  hipStream_t st = hgd::as_stream(stream);
  if (blocks > 0) {
    hipLaunchKernelGGL(hgd::k_adam, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st, L,
                       scalars, step_row, variant);
    hgd_status s = hgd::check_launch("hgd_adam_step");
    if (s != HGD_OK) return s;
  }
  if (step_row) {
    hipLaunchKernelGGL(hgd::k_adam_advance, dim3(1), dim3(1), 0, st, step_row);
    return hgd::check_launch("hgd_adam_step advance");
  }
  return HGD_OK;
}
