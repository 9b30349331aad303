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
//   1. two float4 sweeps of the row: a 2,048-bin histogram of the keys' top 11 bits locates the
//      bin of the K-th largest stream key; the second sweep keeps the keys above that bin and
//      lists the bin's own keys in LDS, whose sort by (key desc, index asc) completes exactly K
//      stream candidates with the lowest-index ties (k_topk_rows). A row whose threshold bin
//      holds more than 2,048 keys (heavy ties) takes the generic path instead: 4 radix passes
//      of 8-bit digits and an ordered compaction (topk_generic);
//   2. bitonic sort of the K candidates and of the K seeds in LDS, merge, write K ids/scores.
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
__device__ __forceinline__ void bitonic_sort(Cand* c, int n) {
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

// Generic path (any score distribution): 4 radix passes over the row for the k-th largest key,
// then an ordered compaction pass. Used when the two-pass path's threshold bin is too full.
__device__ __forceinline__ void topk_generic(const float* __restrict__ row, int64_t n_cols, int k, int* s_hist,
                             int* s_warp, Cand* s_c, int* s_sel) {
  __syncthreads();  // the caller's LDS (histogram) is reused
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
}

// Seeds (the first k entries), sort of the k stream candidates in s_c[0, k) and of the seeds,
// merge: the first k of the union in find_k_largest's order.
__device__ __forceinline__ void topk_finish(const float* __restrict__ row, int k, Cand* s_c, int64_t r,
                            int32_t* __restrict__ out_ids, float* __restrict__ out_scores) {
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

// Two-pass top-k (the common case): pass 1 builds a 2,048-bin histogram of the keys' top 11 bits
// and finds the bin holding the k-th largest; pass 2 appends every key of a higher bin to the
// stream candidates (fewer than k of them, order irrelevant: they are sorted later) and every
// key of the threshold bin (with its index) to an LDS list. Sorting that list by (key desc,
// index asc) and taking its first `need` entries gives exactly the generic path's selection,
// including the lowest-index ties at the k-th key. Two float4 sweeps of the row instead of five
// scalar ones; rows whose threshold bin exceeds kBinCap entries fall back to topk_generic.
constexpr int kHistBins = 2048;
constexpr int kBinCap = 2048;

struct KeyIdx {
  uint32_t key;
  int32_t i;
};

template <typename F>
__device__ __forceinline__ void for_each_score(const float* __restrict__ row, int64_t n_cols,
                                               F f) {
  if ((reinterpret_cast<uintptr_t>(row) & 15) == 0) {
    // kUnroll float4 loads per lane issued before any is consumed (64 B in flight per lane)
    constexpr int kUnroll = 4;
    const float4* r4 = reinterpret_cast<const float4*>(row);
    const int64_t n4 = n_cols >> 2;
    int64_t v0 = 0;
    for (; v0 + kUnroll * kTopkBlock <= n4; v0 += kUnroll * kTopkBlock) {
      float4 x[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) x[u] = r4[v0 + u * kTopkBlock + threadIdx.x];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int64_t c = 4 * (v0 + u * kTopkBlock + threadIdx.x);
        f(x[u].x, c);
        f(x[u].y, c + 1);
        f(x[u].z, c + 2);
        f(x[u].w, c + 3);
      }
    }
    for (int64_t v = v0 + threadIdx.x; v < n4; v += kTopkBlock) {
      const float4 x = r4[v];
      f(x.x, 4 * v);
      f(x.y, 4 * v + 1);
      f(x.z, 4 * v + 2);
      f(x.w, 4 * v + 3);
    }
    for (int64_t c = 4 * n4 + threadIdx.x; c < n_cols; c += kTopkBlock) f(row[c], c);
  } else {
    for (int64_t c = threadIdx.x; c < n_cols; c += kTopkBlock) f(row[c], c);
  }
}

__device__ __forceinline__ bool key_before(const KeyIdx& a, const KeyIdx& b) {
  return a.key != b.key ? a.key > b.key : a.i < b.i;
}

__global__ __launch_bounds__(kTopkBlock) void k_topk_rows(const float* __restrict__ S,
                                                          int64_t n_cols, int64_t ld, int k,
                                                          int32_t* __restrict__ out_ids,
                                                          float* __restrict__ out_scores) {
  __shared__ int s_hist[kHistBins];
  __shared__ int s_warp[kTopkBlock / 64];
  __shared__ Cand s_c[2 * kTopkMax];
  __shared__ KeyIdx s_bin[kBinCap];
  __shared__ int s_sel[4];
  const int64_t r = blockIdx.x;
  const float* row = S + r * ld;

  // pass 1: histogram of the top 11 key bits
  for (int i = threadIdx.x; i < kHistBins; i += kTopkBlock) s_hist[i] = 0;
  __syncthreads();
  int* hist = s_hist;
  for_each_score(row, n_cols, [hist](float s, int64_t) {
    atomicAdd(&hist[float_key(s) >> 21], 1);
  });
  __syncthreads();
  // threshold bin: thread t owns the 8 bins 2047-8t .. 2040-8t (highest first); a block scan
  // of the per-thread counts (high bins first) finds the owner of the k-th largest key
  constexpr int kPer = kHistBins / kTopkBlock;
  const int top = kHistBins - 1 - kPer * threadIdx.x;
  int mine = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) mine += s_hist[top - j];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int incl = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) s_warp[w] = incl;
  __syncthreads();
  for (int i = 0; i < w; ++i) incl += s_warp[i];
  const int excl = incl - mine;
  if (excl < k && incl >= k) {
    int acc = excl, b = top;
    for (;; --b) {
      if (acc + s_hist[b] >= k) break;
      acc += s_hist[b];
    }
    s_sel[0] = b;          // threshold bin
    s_sel[1] = k - acc;    // entries still needed from it
    s_sel[2] = s_hist[b];  // its population
    s_sel[3] = 0;
  }
  __syncthreads();
  const uint32_t sel = static_cast<uint32_t>(s_sel[0]);
  const int need = s_sel[1];
  const int in_bin = s_sel[2];
  const int n_above = k - need;
  if (in_bin > kBinCap) {  // a crowded threshold bin (heavy ties): the generic path
    topk_generic(row, n_cols, k, s_hist, s_warp, s_c, s_sel);
    topk_finish(row, k, s_c, r, out_ids, out_scores);
    return;
  }
  // pass 2: keys of higher bins → stream candidates, threshold-bin keys → s_bin
  if (threadIdx.x == 0) s_hist[0] = 0;  // reused as the two append counters
  if (threadIdx.x == 1) s_hist[1] = 0;
  __syncthreads();
  Cand* cand = s_c;
  KeyIdx* bin = s_bin;
  for_each_score(row, n_cols, [hist, cand, bin, sel](float s, int64_t c) {
    const uint32_t key = float_key(s);
    const uint32_t b = key >> 21;
    if (b > sel) {
      cand[atomicAdd(&hist[0], 1)] = Cand{s, static_cast<int32_t>(c), 0};
    } else if (b == sel) {
      bin[atomicAdd(&hist[1], 1)] = KeyIdx{key, static_cast<int32_t>(c)};
    }
  });
  __syncthreads();
  // sort the threshold bin by (key desc, index asc); its first `need` entries complete the k
  int n2 = 1;
  while (n2 < in_bin) n2 <<= 1;
  for (int t = in_bin + threadIdx.x; t < n2; t += kTopkBlock) s_bin[t] = KeyIdx{0u, 0x7fffffff};
  __syncthreads();
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < n2 / 2; t += kTopkBlock) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool asc = (lo & size) == 0;
        const bool swap = asc ? key_before(s_bin[hi], s_bin[lo]) : key_before(s_bin[lo], s_bin[hi]);
        if (swap) {
          const KeyIdx tmp = s_bin[lo];
          s_bin[lo] = s_bin[hi];
          s_bin[hi] = tmp;
        }
      }
      __syncthreads();
    }
  }
  for (int t = threadIdx.x; t < need; t += kTopkBlock) {
    const int32_t c = s_bin[t].i;
    s_c[n_above + t] = Cand{row[c], c, 0};  // the score itself (keeps the sign of a zero)
  }
  __syncthreads();
  topk_finish(row, k, s_c, r, out_ids, out_scores);
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
