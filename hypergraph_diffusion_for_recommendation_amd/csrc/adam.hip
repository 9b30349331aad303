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
// device buffer the host fills before each launch or graph replay (hgd_adam_scalars), and each
// op's rounding is reproduced in its order. Whether torch's build contracted a multiply-add into
// an fma, and which square root / division it emits, is not visible from Python: `variant` picks
// each (bit 0: lerp fused, bit 1: addcmul fused, bit 2: addcdiv fused, bit 3: fast sqrt, bit 4:
// fast division), and tests/test_gpu_adam.py finds the one that is bitwise torch's on this image.
#include "device_util.h"
#include "hgd_internal.h"

namespace hgd {
namespace {

constexpr int kMaxAdamTensors = 16;

struct AdamList {
  float* p[kMaxAdamTensors];
  const float* g[kMaxAdamTensors];
  float* m[kMaxAdamTensors];
  float* v[kMaxAdamTensors];
  int64_t start[kMaxAdamTensors + 1];  // element offsets of the tensors in the flat index space
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

__global__ __launch_bounds__(256) void k_adam(AdamList L, const float* __restrict__ sc,
                                              int32_t variant) {
#pragma clang fp contract(off)
  const bool f_lerp = variant & 1, f_cmul = variant & 2, f_cdiv = variant & 4;
  const bool fast_sqrt = variant & 8, fast_div = variant & 16;
  const int64_t total = L.start[L.count];
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    int t = 0;
#pragma unroll 1
    while (t + 1 < L.count && i >= L.start[t + 1]) ++t;
    const int64_t e = i - L.start[t];
    const float* s = sc + 6 * t;  // lerp weight, β2, 1 − β2, bias2 sqrt, eps, step size
    const float g = L.g[t][e];
    float m = L.m[t][e];
    float v = L.v[t][e];
    // lerp(m, g, w), w = 1 − β1 < 0.5 (ATen Lerp.h: self + weight·(end − self))
    m = mul_add(s[0], g - m, m, f_lerp);
    // v·β2, then addcmul as torch's foreach pointwise functor: v + value·(g·g)
    v = v * s[1];
    v = mul_add(s[2], g * g, v, f_cmul);
    float d = sqrt_of(v, fast_sqrt);
    d = div_of(d, s[3], fast_div);
    d = d + s[4];
    // addcdiv: p + value·(m / d)
    const float q = div_of(m, d, fast_div);
    L.p[t][e] = mul_add(s[5], q, L.p[t][e], f_cdiv);
    L.m[t][e] = m;
    L.v[t][e] = v;
  }
}

}  // namespace
}  // namespace hgd

extern "C" hgd_status hgd_adam_step(const hgd_adam_tensor* tensors, int32_t count,
                                    const float* scalars, int32_t variant, void* stream) {
  hgd::clear_error();
  HGD_REQUIRE(tensors && count >= 1 && count <= hgd::kMaxAdamTensors,
              "hgd_adam_step: 1 to %d tensors", hgd::kMaxAdamTensors);
  HGD_REQUIRE(scalars, "hgd_adam_step: null scalars");
  HGD_REQUIRE(variant >= 0 && variant < 32, "hgd_adam_step: variant in [0, 32)");
  hgd::AdamList L{};
  L.count = count;
  L.start[0] = 0;
  for (int t = 0; t < count; ++t) {
    const hgd_adam_tensor& x = tensors[t];
    HGD_REQUIRE(x.n >= 0, "hgd_adam_step: tensor %d has a negative size", t);
    HGD_REQUIRE(x.n == 0 || (x.param && x.grad && x.exp_avg && x.exp_avg_sq),
                "hgd_adam_step: tensor %d has a null pointer", t);
    L.p[t] = x.param;
    L.g[t] = x.grad;
    L.m[t] = x.exp_avg;
    L.v[t] = x.exp_avg_sq;
    L.start[t + 1] = L.start[t] + x.n;
  }
  const int64_t total = L.start[count];
  if (total == 0) return HGD_OK;
  const int64_t want = (total + 255) / 256;
  const unsigned blocks = static_cast<unsigned>(want < 4096 ? want : 4096);
  hipLaunchKernelGGL(hgd::k_adam, dim3(blocks), dim3(256), 0, hgd::as_stream(stream), L, scalars,
                     variant);
  return hgd::check_launch("hgd_adam_step");
}
