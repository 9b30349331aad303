// SpAdjDropEdge's keep-mask from torch's CPU generator, bit for bit, without torch's four
// tensor passes.
//
// Reference (paths relative to /root/reference/HD_SELFRec): SpAdjDropEdge.forward
// (model/graph/HCCF.py:217-226 and its copies) draws
//     mask = ((torch.rand(edgeNum) + keepRate).floor()).type(torch.bool)
// on the default CPU generator every layer of every step — at Yelp2018 size 2.3 M draws per
// layer, ≈ 10-30 ms per layer in torch (rand, add, floor, cast, then a count), which bounds the
// whole training step. The same mask comes out of one pass here:
//   * torch's CPU generator is at::mt19937 (MT19937, 32-bit outputs; ATen/core/MT19937RNGEngine.h)
//     and torch.rand(float32) takes one output per element, serially, as
//     ((y & 0xFFFFFF) · 2^-24) (uniform_real_distribution<float>, ATen/core/TransformationHelper.h);
//   * `+ keepRate` adds the float32-rounded scalar in float32, floor(·) != 0  ⇔  sum >= 1.
// The generator state is torch.get_rng_state()'s byte layout (CPUGeneratorImplState: the legacy
// POD with the 624 MT words as uint64, then the float-normal cache), read and written in place
// so the caller hands it back with torch.set_rng_state; the Python side checks the layout once
// against torch.rand itself before using this path.
#include <cstdint>
#include <algorithm>
#include <cstring>

#include "../../include/hgd.h"
#include "hgd_internal.h"

namespace hgd {
namespace {

constexpr int kN = 624;
constexpr int kM = 397;

// torch/csrc (aten/src/ATen/CPUGeneratorImpl.cpp) CPUGeneratorImplStateLegacy + State
struct TorchCpuStateLegacy {
  uint64_t the_initial_seed;
  int32_t left;
  int32_t seeded;
  uint64_t next;
  uint64_t state[kN];
  double normal_x;
  double normal_y;
  double normal_rho;
  int32_t normal_is_valid;
};
struct TorchCpuState {
  TorchCpuStateLegacy legacy_pod;
  float next_float_normal_sample;
  bool is_next_float_normal_sample_valid;
};
static_assert(sizeof(TorchCpuState) == 5056, "torch CPU generator state layout");

__attribute__((always_inline)) inline uint32_t twist(uint32_t u, uint32_t v) {
  return (((u & 0x80000000u) | (v & 0x7fffffffu)) >> 1) ^ ((v & 1u) ? 0x9908b0dfu : 0u);
}

// at::mt19937::next_state on a plain uint32 array
__attribute__((always_inline)) inline void next_state(uint32_t* s) {
  uint32_t* p = s;
  for (int j = kN - kM + 1; --j; ++p) *p = p[kM] ^ twist(p[0], p[1]);
  for (int j = kM; --j; ++p) *p = p[kM - kN] ^ twist(p[0], p[1]);
  *p = p[kM - kN] ^ twist(p[0], s[0]);
}

__attribute__((always_inline)) inline uint32_t temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

// The draw loop, shared by the AVX2 and the baseline build of it (selected at run time): the
// tempering / compare loop and both halves of the state refill auto-vectorise.
struct Draws {
  uint32_t s[kN];
  int left;
  uint32_t next;
};

__attribute__((always_inline)) inline int64_t draw_mask(Draws& g, int64_t n, float keep,
                                                        uint8_t* mask) {
  int64_t cnt = 0;
  int64_t k = 0;
  while (k < n) {
    // at::mt19937::operator(): if (--left == 0) next_state(); y = state[next++]
    if (--g.left == 0) {
      next_state(g.s);
      g.left = kN;
      g.next = 0;
    }
    // calls that succeed before the next refill: `left` of them (this one included), each
    // consuming s[next++]
    const int64_t run = std::min<int64_t>(n - k, g.left);
    const uint32_t* src = g.s + g.next;
    uint8_t* dst = mask + k;
    int64_t c = 0;
    for (int64_t t = 0; t < run; ++t) {
      const uint32_t y = temper(src[t]);
      const float r = static_cast<float>(y & 0xFFFFFFu) * (1.0f / 16777216.0f);
      const float v = r + keep;              // float32 add, as the tensor op
      const uint8_t m = v >= 1.0f ? 1 : 0;   // floor(v) != 0 for v in [keep, keep + 1)
      dst[t] = m;
      c += m;
    }
    cnt += c;
    g.next += static_cast<uint32_t>(run);
    g.left -= static_cast<int>(run - 1);  // the first call of the run already decremented
    k += run;
  }
  return cnt;
}

__attribute__((target("avx2"))) int64_t draw_mask_avx2(Draws& g, int64_t n, float keep,
                                                       uint8_t* mask) {
  return draw_mask(g, n, keep, mask);
}

int64_t draw_mask_base(Draws& g, int64_t n, float keep, uint8_t* mask) {
  return draw_mask(g, n, keep, mask);
}

}  // namespace
}  // namespace hgd

extern "C" size_t hgd_torch_cpu_state_bytes(void) { return sizeof(hgd::TorchCpuState); }

extern "C" hgd_status hgd_torch_cpu_keep_mask(uint8_t* torch_state, int64_t state_bytes,
                                              int64_t n, float keep, uint8_t* mask,
                                              int64_t* kept) {
  using namespace hgd;
  clear_error();
  HGD_REQUIRE(torch_state && state_bytes == static_cast<int64_t>(sizeof(TorchCpuState)),
              "hgd_torch_cpu_keep_mask: state must be the %zu bytes of torch.get_rng_state()",
              sizeof(TorchCpuState));
  HGD_REQUIRE(n >= 0 && (mask || n == 0), "hgd_torch_cpu_keep_mask: bad n / mask");
  TorchCpuState st;
  std::memcpy(&st, torch_state, sizeof(st));
  TorchCpuStateLegacy& L = st.legacy_pod;
  HGD_REQUIRE(L.left >= 1 && L.left <= kN && L.next <= static_cast<uint64_t>(kN),
              "hgd_torch_cpu_keep_mask: generator state out of range (left=%d next=%llu)",
              L.left, static_cast<unsigned long long>(L.next));
  Draws g;
  for (int i = 0; i < kN; ++i) g.s[i] = static_cast<uint32_t>(L.state[i]);
  g.left = L.left;
  g.next = static_cast<uint32_t>(L.next);
  static const bool avx2 = __builtin_cpu_supports("avx2");
  const int64_t cnt = n == 0 ? 0 : (avx2 ? draw_mask_avx2(g, n, keep, mask)
                                         : draw_mask_base(g, n, keep, mask));
  for (int i = 0; i < kN; ++i) L.state[i] = g.s[i];
  L.left = g.left;
  L.next = g.next;
  std::memcpy(torch_state, &st, sizeof(st));
  if (kept) *kept = cnt;
  return HGD_OK;
}
