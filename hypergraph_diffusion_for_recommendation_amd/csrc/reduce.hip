// Deterministic column sums of a partials matrix P [S, W] (hgd_internal.h: sum_rows).
//
// The serial form (one thread per column walking all S rows) is a chain of S dependent-latency
// loads — 0.25 ms at S = 1024 in profiles/r01_edhnn_yelp. Here a 1024-thread block owns 64
// columns; each of its 16 waves sums a contiguous 1/16 of the rows with 8 loads in flight, and
// the 16 wave sums are added in wave order, so the result is independent of timing.
#include "hgd_internal.h"

namespace hgd {
namespace {

constexpr int kWaves = 16;

struct Jobs {
  SumRowsJob j[4];
  int64_t first[5];  // first block of each job
  int n;
};

__global__ __launch_bounds__(kWaves * 64) void k_sum_rows(Jobs jobs) {
  __shared__ float s_part[kWaves][64];
  int ji = 0;
  for (int k = 1; k < jobs.n; ++k) ji += static_cast<int64_t>(blockIdx.x) >= jobs.first[k];
  const SumRowsJob J = jobs.j[ji];
  const float* __restrict__ P = J.P;
  const int64_t S = J.S, W = J.W;
  float* __restrict__ out = J.out;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t c = (static_cast<int64_t>(blockIdx.x) - jobs.first[ji]) * 64 + lane;
  const int64_t per = (S + kWaves - 1) / kWaves;
  const int64_t s0 = w * per;
  const int64_t s1 = s0 + per < S ? s0 + per : S;
  float acc = 0.f;
  if (c < W) {
    int64_t s = s0;
    for (; s + 8 <= s1; s += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = P[(s + u) * W + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; s < s1; ++s) acc += P[s * W + c];
  }
  s_part[w][lane] = acc;
  __syncthreads();
  if (w != 0 || c >= W) return;
  float t = s_part[0][lane];
#pragma unroll
  for (int k = 1; k < kWaves; ++k) t += s_part[k][lane];
  out[c] = J.scale != 0.f ? t * J.scale : t;
}

}  // namespace

hgd_status sum_rows_jobs(const SumRowsJob* js, int n, hipStream_t st) {
  Jobs jobs{};
  int64_t blocks = 0;
  for (int i = 0; i < n; ++i) {
    if (js[i].W <= 0) continue;
    jobs.first[jobs.n] = blocks;
    jobs.j[jobs.n++] = js[i];
    blocks += (js[i].W + 63) / 64;
  }
  if (jobs.n == 0) return HGD_OK;
  jobs.first[jobs.n] = blocks;
  if (blocks > 0x7fffffffLL) return fail(HGD_ERR_UNSUPPORTED, "sum_rows: too many columns");
  hipLaunchKernelGGL(k_sum_rows, dim3(blocks), dim3(kWaves * 64), 0, st, jobs);
  return check_launch("sum_rows");
}

hgd_status sum_rows(const float* P, int64_t S, int64_t W, float* out, hipStream_t st) {
  const SumRowsJob j{P, S, W, out, 0.f};
  return sum_rows_jobs(&j, 1, st);
}

}  // namespace hgd
