// Batched top-K recommendation lists with the reference's exact selection semantics.
//
// Reference (paths relative to /root/reference/HD_SELFRec): GraphRecommender.test()
// (base/graph_recommender.py:61-92) scores one user at a time (predict: user_emb[u]·item_embᵀ),
// sets every rated item to -10e8 (:79-80) and calls numba find_k_largest(K, candidates)
// (util/algorithm.py:143-173). find_k_largest seeds its list with candidates[:K] sorted
// descending (stable), then streams ALL candidates again (iid = 0..n-1), inserting a candidate
// when it is strictly larger than the current K-th score, after every entry with an equal or
// larger score. Closed form: the result is the first K entries of
//     seed = {(c_j, j) : j < K}  ∪  stream = {(c_i, i) : i < n}
// ordered by score descending, then seed before stream, then index ascending — which is why an
// item among the first K with a top score is listed twice by the reference, and is here too.
//
// GPU mapping (one 256-thread workgroup per score row, rows are HBM-streamed):
//   1. radix select of the K-th largest stream key (4 passes of 8-bit digits, LDS histogram);
//   2. ordered compaction: every key above the threshold plus the lowest-index ties, giving
//      exactly K stream candidates (block-wide prefix sums keep index order);
//   3. bitonic sort of the K candidates and of the K seeds in LDS, merge, write K ids/scores.
// Masking is a separate scatter (hgd_mask_scores) that writes the reference's -10e8 in place.
#include "hgd_internal.h"

namespace hgd {

constexpr int kTopkBlock = 256;
constexpr int kTopkMax = 256;  // K <= 256 (the reference's item_ranking tops out at 40)

__device__ __forceinline__ uint32_t float_key(float f) {
  if (f == 0.f) f = 0.f;  // -0.0 and +0.0 compare equal in the reference: one key
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Block-wide exclusive prefix over one 0/1 flag per thread (thread order = index order).
__device__ __forceinline__ int block_excl_prefix(bool flag, int* s_warp, int& total) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const unsigned long long b = __ballot(flag);
  const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  const int in_wave = __popcll(b & lt);
  if (lane == 0) s_warp[w] = __popcll(b);
  __syncthreads();
  int base = 0;
  total = 0;
  for (int i = 0; i < kTopkBlock / 64; ++i) {
    if (i < w) base += s_warp[i];
    total += s_warp[i];
  }
  __syncthreads();
  return base + in_wave;
}

struct Cand {
  float s;
  int32_t i;
  int32_t seed;  // 1 = seed copy (precedes stream entries of equal score)
};

// a before b in the output order
__device__ __forceinline__ bool cand_before(const Cand& a, const Cand& b) {
  if (a.s != b.s) return a.s > b.s;
  if (a.seed != b.seed) return a.seed > b.seed;
  return a.i < b.i;
}

// In-LDS bitonic sort of n (power of two, <= 2*kTopkBlock) candidates, best first.
__device__ void bitonic_sort(Cand* c, int n) {
  for (int size = 2; size <= n; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < n / 2; t += kTopkBlock) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool asc = (lo & size) == 0;  // "ascending" = best first in this sub-sequence
        const bool swap = asc ? cand_before(c[hi], c[lo]) : cand_before(c[lo], c[hi]);
        if (swap) {
          const Cand tmp = c[lo];
          c[lo] = c[hi];
          c[hi] = tmp;
        }
      }
      __syncthreads();
    }
  }
}

__global__ __launch_bounds__(kTopkBlock) void k_topk_rows(const float* __restrict__ S,
                                                          int64_t n_cols, int64_t ld, int k,
                                                          int32_t* __restrict__ out_ids,
                                                          float* __restrict__ out_scores) {
  __shared__ int s_hist[256];
  __shared__ int s_warp[kTopkBlock / 64];
  __shared__ Cand s_c[2 * kTopkMax];
  __shared__ int s_sel[2];
  const int64_t r = blockIdx.x;
  const float* row = S + r * ld;

  // 1. radix select: the k-th largest key of the row
  uint32_t prefix = 0, pmask = 0;
  int need = k;  // rank (1-based) still to find inside the current prefix class
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = threadIdx.x; i < 256; i += kTopkBlock) s_hist[i] = 0;
    __syncthreads();
    for (int64_t c = threadIdx.x; c < n_cols; c += kTopkBlock) {
      const uint32_t key = float_key(row[c]);
      if ((key & pmask) == prefix) atomicAdd(&s_hist[(key >> shift) & 255], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int acc = 0, digit = 255;
      for (; digit > 0; --digit) {
        if (acc + s_hist[digit] >= need) break;
        acc += s_hist[digit];
      }
      s_sel[0] = digit;
      s_sel[1] = need - acc;
    }
    __syncthreads();
    prefix |= static_cast<uint32_t>(s_sel[0]) << shift;
    pmask |= 255u << shift;
    need = s_sel[1];
    __syncthreads();
  }
  const uint32_t thr = prefix;  // key of the k-th largest; `need` ties of it are taken

  // 2. ordered compaction: keys > thr, then the first `need` keys == thr in index order
  int n_above = 0, n_ties = 0;
  for (int64_t c0 = 0; c0 < n_cols; c0 += kTopkBlock) {
    const int64_t c = c0 + threadIdx.x;
    float s = 0.f;
    uint32_t key = 0;
    if (c < n_cols) {
      s = row[c];
      key = float_key(s);
    }
    const bool above = c < n_cols && key > thr;
    const bool tie = c < n_cols && key == thr;
    int tot_a, tot_t;
    const int pa = block_excl_prefix(above, s_warp, tot_a);
    const int pt = block_excl_prefix(tie, s_warp, tot_t);
    if (above) s_c[n_above + pa] = Cand{s, static_cast<int32_t>(c), 0};
    if (tie && n_ties + pt < need)
      s_c[(k - need) + n_ties + pt] = Cand{s, static_cast<int32_t>(c), 0};
    n_above += tot_a;
    n_ties += tot_t;
    __syncthreads();
  }
  // 3. seeds, sort both halves, merge (first k of the union)
  int n2 = 1;
  while (n2 < k) n2 <<= 1;
  for (int t = threadIdx.x; t < n2; t += kTopkBlock) {
    if (t < k) {
      s_c[kTopkMax + t] = Cand{row[t], t, 1};
    } else {
      s_c[t] = Cand{-INFINITY, 0x7fffffff, 0};
      s_c[kTopkMax + t] = Cand{-INFINITY, 0x7fffffff, 0};
    }
  }
  __syncthreads();
  bitonic_sort(s_c, n2);
  bitonic_sort(s_c + kTopkMax, n2);
  if (threadIdx.x == 0) {
    int a = 0, b = 0;
    for (int o = 0; o < k; ++o) {
      const Cand& x = s_c[a];
      const Cand& y = s_c[kTopkMax + b];
      const bool take_seed = cand_before(y, x);
      const Cand& z = take_seed ? y : x;
      out_ids[r * k + o] = z.i;
      out_scores[r * k + o] = z.s;
      if (take_seed)
        ++b;
      else
        ++a;
    }
  }
}

// S[r, cols of mask row m(r)] = value, m(r) = row_map ? row_map[r] : r.
__global__ void k_mask_scores(float* __restrict__ S, int64_t n_rows, int64_t ld,
                              const int64_t* __restrict__ rowptr,
                              const int32_t* __restrict__ cols,
                              const int32_t* __restrict__ row_map, float value) {
  const int64_t r = blockIdx.x;
  if (r >= n_rows) return;
  const int64_t m = row_map ? row_map[r] : r;
  for (int64_t e = rowptr[m] + threadIdx.x; e < rowptr[m + 1]; e += blockDim.x)
    S[r * ld + cols[e]] = value;
}

}  // namespace hgd

using namespace hgd;

extern "C" hgd_status hgd_mask_scores(float* scores, int64_t n_rows, int64_t ld,
                                      const int64_t* rowptr, const int32_t* cols,
                                      const int32_t* row_map, float value, void* stream) {
  clear_error();
  HGD_REQUIRE(n_rows >= 0 && ld > 0, "hgd_mask_scores: sizes");
  if (n_rows == 0) return HGD_OK;
  HGD_REQUIRE(scores && rowptr, "hgd_mask_scores: null pointer");
  if (n_rows > 0x7fffffffLL) return fail(HGD_ERR_UNSUPPORTED, "hgd_mask_scores: too many rows");
  hipLaunchKernelGGL(k_mask_scores, dim3(n_rows), dim3(64), 0, as_stream(stream), scores, n_rows,
                     ld, rowptr, cols, row_map, value);
  return check_launch("hgd_mask_scores");
}

extern "C" hgd_status hgd_topk_rows(const float* scores, int64_t n_rows, int64_t n_cols, int64_t ld,
                                    int32_t k, int32_t* out_ids, float* out_scores,
                                    void* stream) {
  clear_error();
  HGD_REQUIRE(n_rows >= 0 && n_cols >= 0 && ld >= n_cols, "hgd_topk_rows: sizes");
  HGD_REQUIRE(k >= 1 && k <= kTopkMax, "hgd_topk_rows: k must be in [1, %d]", kTopkMax);
  HGD_REQUIRE(n_cols >= k, "hgd_topk_rows: fewer columns (%lld) than k (%d)",
              (long long)n_cols, k);
  if (n_rows == 0) return HGD_OK;
  HGD_REQUIRE(scores && out_ids && out_scores, "hgd_topk_rows: null pointer");
  if (n_rows > 0x7fffffffLL) return fail(HGD_ERR_UNSUPPORTED, "hgd_topk_rows: too many rows");
  hipLaunchKernelGGL(k_topk_rows, dim3(n_rows), dim3(kTopkBlock), 0, as_stream(stream), scores,
                     n_cols, ld, k, out_ids, out_scores);
  return check_launch("hgd_topk_rows");
}
