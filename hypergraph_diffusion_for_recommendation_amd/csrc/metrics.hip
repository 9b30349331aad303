// Per-user ranking metrics of the top-K lists, with the reference's exact arithmetic.
//
// Reference (paths relative to /root/reference/HD_SELFRec): ranking_evaluation
// (util/evaluation.py:169-196) cuts every user's list at each N of item_ranking and calls
//   Metric.hits  (:8-15)   |set(test items) ∩ set(predicted[:N])|  — DISTINCT predicted names, so
//                          an item find_k_largest lists twice (topk.hip) counts once;
//   Metric.NDCG  (:84-97)  DCG = Σ_{n < N, predicted[n] in test} 1.0/math.log(n+2, 2), summed in
//                          position order (a duplicated hit contributes at both positions).
// Those two per-user quantities are what this kernel produces; the remaining arithmetic of the
// reference (IDCG from the test-set size, recall = hits/|test|, the dataset sums in test_set order,
// round(·, 5)) is done by the host in the reference's order (evaluation.ranking_evaluation).
//
// The discount 1/log(n+2, 2) is taken as a host-computed float64 table (the reference's
// math.log(x, 2) = log(x)/log(2), not log2), and DCG is accumulated sequentially in position order
// in float64, so the per-user DCG is bit-identical to the reference loop.
//
// Mapping: one wave per user row (the row is ≤ 256 ids). The row's ids go to LDS; each lane
// tests its positions against the user's sorted test list (binary search) and against the earlier
// positions of the row (first occurrence, for the set semantics); two ballots per 64 positions
// hand the flags to lane 0, which walks the positions in order, emitting (hits, DCG) at every
// cut-off. K ids + the test list per user: tiny, latency-bound work.
#include "hgd_internal.h"

namespace hgd {
namespace {

constexpr int kMetricsMaxK = 256;
constexpr int kMetricsMaxCut = 16;
constexpr int kWavesPerBlock = kBlock / 64;

struct Cutoffs {
  int32_t n;
  int32_t at[kMetricsMaxCut];  // ascending, each in [1, k]
};

__device__ __forceinline__ bool in_sorted(const int32_t* a, int64_t lo, int64_t hi, int32_t v) {
  while (lo < hi) {
    const int64_t mid = lo + ((hi - lo) >> 1);
    const int32_t x = a[mid];
    if (x == v) return true;
    if (x < v)
      lo = mid + 1;
    else
      hi = mid;
  }
  return false;
}

__global__ __launch_bounds__(kBlock) void k_rank_metrics(
    const int32_t* __restrict__ ids, int64_t n_rows, int64_t ld, int k,
    const int64_t* __restrict__ trowptr, const int32_t* __restrict__ tcols, Cutoffs cut,
    const double* __restrict__ disc, int32_t* __restrict__ hits, double* __restrict__ dcg) {
  __shared__ int32_t s_ids[kWavesPerBlock][kMetricsMaxK];
  const int w = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kWavesPerBlock + w;
  if (r >= n_rows) return;  // wave-uniform; only wave-level synchronisation below
  const int32_t* row = ids + r * ld;
  for (int p = lane; p < k; p += 64) s_ids[w][p] = row[p];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int64_t t0 = trowptr[r], t1 = trowptr[r + 1];
  const int n_cut = cut.n;

  int hc = 0;      // lane 0: distinct hits so far
  double d = 0.0;  // lane 0: DCG so far (position order)
  int ci = 0;      // lane 0: next cut-off to emit
  for (int base = 0; base < k; base += 64) {
    const int p = base + lane;
    bool in = false, first = false;
    if (p < k) {
      const int32_t id = s_ids[w][p];
      in = id >= 0 && in_sorted(tcols, t0, t1, id);
      if (in) {
        first = true;
        for (int q = 0; q < p; ++q)
          if (s_ids[w][q] == id) {
            first = false;
            break;
          }
      }
    }
    const unsigned long long m_in = __ballot(in);
    const unsigned long long m_first = __ballot(first);
    if (lane == 0) {
      const int nb = min(64, k - base);
      for (int j = 0; j < nb; ++j) {
        const int pos = base + j;
        while (ci < n_cut && cut.at[ci] == pos) {  // predicted[:N] = positions < N
          hits[r * n_cut + ci] = hc;
          dcg[r * n_cut + ci] = d;
          ++ci;
        }
        if ((m_in >> j) & 1ull) d += disc[pos];
        if ((m_first >> j) & 1ull) ++hc;
      }
    }
  }
  if (lane == 0) {
    while (ci < n_cut) {  // cut-offs equal to k
      hits[r * n_cut + ci] = hc;
      dcg[r * n_cut + ci] = d;
      ++ci;
    }
  }
}

}  // namespace
}  // namespace hgd

extern "C" hgd_status hgd_rank_metrics(const int32_t* ids, int64_t n_rows, int64_t ld, int32_t k,
                                       const int64_t* test_rowptr, const int32_t* test_cols,
                                       const int32_t* cutoffs, int32_t n_cutoffs,
                                       const double* discount, int32_t* hits, double* dcg,
                                       void* stream) {
  using namespace hgd;
  clear_error();
  HGD_REQUIRE(k >= 1 && k <= kMetricsMaxK, "hgd_rank_metrics: k must be in [1, %d] (got %d)",
              kMetricsMaxK, k);
  HGD_REQUIRE(n_rows >= 0 && ld >= k, "hgd_rank_metrics: bad n_rows / ld");
  HGD_REQUIRE(cutoffs && n_cutoffs >= 1 && n_cutoffs <= kMetricsMaxCut,
              "hgd_rank_metrics: need 1..%d cut-offs (got %d)", kMetricsMaxCut, n_cutoffs);
  Cutoffs cut{};
  cut.n = n_cutoffs;
  for (int i = 0; i < n_cutoffs; ++i) {
    HGD_REQUIRE(cutoffs[i] >= 1 && cutoffs[i] <= k && (i == 0 || cutoffs[i] > cutoffs[i - 1]),
                "hgd_rank_metrics: cut-offs must be ascending in [1, k=%d] (cutoffs[%d]=%d)", k,
                i, cutoffs[i]);
    cut.at[i] = cutoffs[i];
  }
  if (n_rows == 0) return HGD_OK;
  HGD_REQUIRE(ids && test_rowptr && discount && hits && dcg, "hgd_rank_metrics: null pointer");
  const int64_t blocks = (n_rows + kWavesPerBlock - 1) / kWavesPerBlock;
  HGD_REQUIRE(blocks <= 0x7fffffffLL, "hgd_rank_metrics: too many rows");
  hipLaunchKernelGGL(k_rank_metrics, dim3(static_cast<unsigned>(blocks)), dim3(kBlock), 0,
                     as_stream(stream), ids, n_rows, ld, static_cast<int>(k), test_rowptr,
                     test_cols, cut, discount, hits, dcg);
  return check_launch("hgd_rank_metrics");
}
