// Structure primitives feeding the SpMM hops: COO→CSR ordering, CSR→CSC transpose support,
// degree scales, per-nonzero weights, drop-edge compaction and dense-threshold nonzero.
// All outputs are deterministic and bit-exact with the CPU restatement in oracle/.
//
// Reference behaviour restated (paths relative to /root/reference/HD_SELFRec):
//   rowptr / sort      base/torch_interface.py:8-12 (row-major COO), cuSPARSE coalesce inside
//                      torch.sparse.mm and the `adj.t()` transpose of HGCNConv (HGNN_HD4.py:459)
//   degree scale       data/graph.py:11-25 (D^-1/2 A D^-1/2, D^-1 A, inf→0), data/graph.py:28-42
//   drop-edge          model/graph/HCCF.py:213-226 (mask → idxs[:,mask], vals[mask]/keepRate)
//   dense threshold    model/layers/layers2/EquivSetGNN2.py:105-133 (torch.nonzero(H > 0))
#include <hipcub/hipcub.hpp>

#include "device_util.h"
#include "hgd_internal.h"

namespace hgd {

thread_local char g_last_error[512] = {0};

// ------------------------------------------------------------------------------------------
__global__ void k_plan_count(const int64_t* __restrict__ rowptr, int64_t n_rows,
                             int64_t threshold, int32_t chunk,
                             unsigned long long* __restrict__ counts) {
  __shared__ unsigned long long s_h[kBlock / 64], s_c[kBlock / 64];
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  unsigned long long h = 0, c = 0;
  if (r < n_rows) {
    const int64_t deg = rowptr[r + 1] - rowptr[r];
    if (deg > threshold) {
      h = 1;
      c = static_cast<unsigned long long>((deg + chunk - 1) / chunk);
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    h += __shfl_down(h, off, 64);
    c += __shfl_down(c, off, 64);
  }
  const int w = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) {
    s_h[w] = h;
    s_c[w] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long th = 0, tc = 0;
    for (int i = 0; i < kBlock / 64; ++i) {
      th += s_h[i];
      tc += s_c[i];
    }
    if (th) atomicAdd(&counts[0], th);
    if (tc) atomicAdd(&counts[1], tc);
  }
}

__global__ void k_plan_flags(const int64_t* __restrict__ rowptr, int64_t n_rows,
                             int64_t threshold, int32_t chunk, int64_t* __restrict__ flag,
                             int64_t* __restrict__ nch) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (r > n_rows) return;
  int64_t f = 0, c = 0;
  if (r < n_rows) {
    const int64_t deg = rowptr[r + 1] - rowptr[r];
    if (deg > threshold) {
      f = 1;
      c = (deg + chunk - 1) / chunk;
    }
  }
  flag[r] = f;  // entry n_rows is 0 so the exclusive scan leaves the total there
  nch[r] = c;
}

__global__ void k_plan_scatter(const int64_t* __restrict__ rowptr, int64_t n_rows,
                               int64_t threshold, const int64_t* __restrict__ pos,
                               const int64_t* __restrict__ cpos, int32_t* __restrict__ heavy_rows,
                               int64_t* __restrict__ heavy_cptr, int64_t n_heavy) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (r > n_rows) return;
  if (r == n_rows) {
    heavy_cptr[n_heavy] = cpos[n_rows];
    return;
  }
  if (rowptr[r + 1] - rowptr[r] > threshold) {
    const int64_t p = pos[r];
    heavy_rows[p] = static_cast<int32_t>(r);
    heavy_cptr[p] = cpos[r];
  }
}

__global__ void k_plan_chunks(const int64_t* __restrict__ heavy_cptr, int64_t n_heavy,
                              int64_t n_chunks, int32_t* __restrict__ chunk_heavy) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (t >= n_chunks) return;
  // largest h with heavy_cptr[h] <= t
  int64_t lo = 0, hi = n_heavy;  // invariant: heavy_cptr[lo] <= t < heavy_cptr[hi]
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (heavy_cptr[mid] <= t)
      lo = mid;
    else
      hi = mid;
  }
  chunk_heavy[t] = static_cast<int32_t>(lo);
}

// ------------------------------------------------------------------------------------------
__global__ void k_index_narrow(const int64_t* __restrict__ in, int64_t n, int64_t upper,
                               int32_t* __restrict__ out, unsigned long long* err) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  const int64_t v = in[i];
  const bool bad = v < 0 || v >= upper;
  out[i] = bad ? 0 : static_cast<int32_t>(v);
  if (bad) atomicAdd(err, 1ull);
}

__global__ void k_iota(int32_t* __restrict__ out, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) out[i] = static_cast<int32_t>(i);
}

__global__ void k_rowptr_from_sorted(const int32_t* __restrict__ rows, int64_t nnz,
                                     int64_t n_rows, int64_t* __restrict__ rowptr) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (r > n_rows) return;
  int64_t lo = 0, hi = nnz;  // first p with rows[p] >= r
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (rows[mid] < r)
      lo = mid + 1;
    else
      hi = mid;
  }
  rowptr[r] = lo;
}

__global__ void k_check_sorted(const int32_t* __restrict__ rows, int64_t nnz, int64_t n_rows,
                               unsigned long long* bad) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (e >= nnz) return;
  const int32_t v = rows[e];
  bool b = v < 0 || v >= n_rows;
  if (e > 0 && rows[e - 1] > v) b = true;
  if (b) atomicAdd(bad, 1ull);
}

__global__ void k_expand_rows(const int64_t* __restrict__ rowptr, int64_t n_rows,
                              int32_t* __restrict__ rows_out, int64_t nnz) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (e >= nnz) return;
  int64_t lo = 0, hi = n_rows;  // last r with rowptr[r] <= e
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (rowptr[mid] <= e)
      lo = mid;
    else
      hi = mid;
  }
  rows_out[e] = static_cast<int32_t>(lo);
}

__global__ void k_gather32(const uint32_t* __restrict__ src, const int32_t* __restrict__ perm,
                           int64_t n, uint32_t* __restrict__ out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) out[i] = src[perm[i]];
}

// out[i] = src[perm[i]] for bytes (a keep-mask into the other orientation's edge order): four
// outputs per thread, so the permutation is read as one 16-byte load and the output written as
// one 4-byte store.
__global__ void k_gather_u8(const uint8_t* __restrict__ src, const int32_t* __restrict__ perm,
                            int64_t n, uint8_t* __restrict__ out) {
  const int64_t i = 4 * (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x);
  if (i + 4 <= n) {
    const int4 p = *reinterpret_cast<const int4*>(perm + i);
    const uint32_t v = static_cast<uint32_t>(src[p.x]) | (static_cast<uint32_t>(src[p.y]) << 8) |
                       (static_cast<uint32_t>(src[p.z]) << 16) |
                       (static_cast<uint32_t>(src[p.w]) << 24);
    *reinterpret_cast<uint32_t*>(out + i) = v;
  } else {
    for (int64_t j = i; j < n; ++j) out[j] = src[perm[j]];
  }
}

__global__ void k_degree_scale(const int64_t* __restrict__ rowptr, const float* __restrict__ val,
                               int64_t n_rows, double power, float* __restrict__ out) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (r >= n_rows) return;
  double deg;
  if (val) {
    float s = 0.f;  // fp32 row sum in edge order (scipy sums the float32 matrix in float32)
    for (int64_t e = rowptr[r]; e < rowptr[r + 1]; ++e) s += val[e];
    deg = static_cast<double>(s);
  } else {
    deg = static_cast<double>(rowptr[r + 1] - rowptr[r]);
  }
  float res;
  if (deg == 0.0) {
    res = 0.f;  // np.power(0, -p) = inf → 0 (data/graph.py:16)
  } else if (power == -1.0) {
    res = static_cast<float>(1.0 / deg);
  } else if (power == -0.5) {
    res = static_cast<float>(1.0 / sqrt(deg));
  } else {
    res = static_cast<float>(pow(deg, power));
  }
  out[r] = res;
}

__global__ void k_edge_values(const float* __restrict__ base, const int32_t* __restrict__ perm,
                              const float* __restrict__ src_scale,
                              const int32_t* __restrict__ src_idx, int64_t n,
                              float* __restrict__ out) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (e >= n) return;
  float v = 1.f;
  if (base) v = base[perm ? perm[e] : e];
  if (src_scale) v *= src_scale[src_idx[e]];
  out[e] = v;
}

// ---- ordered stream compaction, reduce-then-scan over tiles ----------------------------------
// The drop-edge paths keep the entries whose flag is set, in order. A device-wide scan of one
// flag per entry (hipcub DeviceScan, decoupled lookback over ~n/2048 blocks) costs a serial
// chain of block-to-block handoffs — 27 µs for 2.3 M entries, 20x the bytes it moves. Here:
// k_tile_count counts each 2,048-entry tile, k_tile_scan (one block) turns the counts into tile
// offsets, and k_tile_compact recomputes the flags and writes every kept entry at
// tile offset + its in-tile prefix (wave ballots + a 4-wave LDS prefix per 256-entry round).
constexpr int kTileThreads = 256;
constexpr int kTileIter = 8;
constexpr int64_t kTile = static_cast<int64_t>(kTileThreads) * kTileIter;

struct MaskFlag {  // entry e kept iff mask[perm ? perm[e] : e] != 0
  const uint8_t* mask;
  const int32_t* perm;
  __device__ bool operator()(int64_t e) const { return mask[perm ? perm[e] : e] != 0; }
};

struct StructWriter {  // one orientation: idx_out[p] = idx[e], val_out[p] = val[e] / keep
  const int32_t* idx;
  const float* val;
  float keep;
  int32_t* idx_out;
  float* val_out;
  __device__ void operator()(int64_t e, int64_t p) const {
    idx_out[p] = idx[e];
    if (val) val_out[p] = __fdiv_rn(val[e], keep);  // IEEE fp32 division like vals / keepRate
  }
};

struct CooWriter {  // idxs[:, mask], vals[mask] / keepRate
  const int64_t* rows;
  const int64_t* cols;
  const float* val;
  float keep;
  int64_t* out_rows;
  int64_t* out_cols;
  float* out_val;
  __device__ void operator()(int64_t e, int64_t p) const {
    out_rows[p] = rows[e];
    out_cols[p] = cols[e];
    out_val[p] = __fdiv_rn(val[e], keep);
  }
};

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

template <class F>
__global__ __launch_bounds__(kTileThreads) void k_tile_count(F flag, int64_t n,
                                                            int32_t* __restrict__ tile_cnt) {
  __shared__ int s_w[kTileThreads / 64];
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kTile;
  int c = 0;
#pragma unroll
  for (int j = 0; j < kTileIter; ++j) {
    const int64_t e = base + j * kTileThreads + threadIdx.x;
    c += (e < n && flag(e)) ? 1 : 0;
  }
  c = wave_sum_i(c);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < kTileThreads / 64; ++w) t += s_w[w];
    tile_cnt[blockIdx.x] = t;
  }
}

// One block: off[t] = Σ_{t' < t} cnt[t'] for t <= n_tiles (off[n_tiles] = total).
__global__ __launch_bounds__(1024) void k_tile_scan(const int32_t* __restrict__ cnt,
                                                   int64_t n_tiles, int64_t* __restrict__ off) {
  __shared__ int64_t s[1024];
  const int64_t per = (n_tiles + 1023) / 1024;
  const int64_t t0 = static_cast<int64_t>(threadIdx.x) * per;
  const int64_t t1 = t0 + per < n_tiles ? t0 + per : n_tiles;
  int64_t sum = 0;
  for (int64_t t = t0; t < t1; ++t) sum += cnt[t];
  s[threadIdx.x] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const int64_t v = static_cast<int>(threadIdx.x) >= d ? s[threadIdx.x - d] : 0;
    __syncthreads();
    s[threadIdx.x] += v;
    __syncthreads();
  }
  int64_t run = s[threadIdx.x] - sum;
  for (int64_t t = t0; t < t1; ++t) {
    off[t] = run;
    run += cnt[t];
  }
  if (threadIdx.x == 1023) off[n_tiles] = s[1023];
}

template <class F, class W>
__global__ __launch_bounds__(kTileThreads) void k_tile_compact(F flag, W write, int64_t n,
                                                              const int64_t* __restrict__ tile_off,
                                                              int32_t* __restrict__ pos_in_tile) {
  __shared__ int s_w[kTileThreads / 64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kTile;
  const int64_t off = tile_off[blockIdx.x];
  int in_tile = 0;
  for (int j = 0; j < kTileIter; ++j) {
    const int64_t e = base + j * kTileThreads + threadIdx.x;
    const bool f = e < n && flag(e);
    const unsigned long long ball = __ballot(f);
    const int before = __popcll(ball & ((1ull << lane) - 1ull));
    if (lane == 0) s_w[wave] = __popcll(ball);
    __syncthreads();
    int wave_off = 0, round = 0;
#pragma unroll
    for (int w = 0; w < kTileThreads / 64; ++w) {
      wave_off += w < wave ? s_w[w] : 0;
      round += s_w[w];
    }
    const int my = in_tile + wave_off + before;  // kept entries of this tile before e
    if (pos_in_tile && e < n) pos_in_tile[e] = my;
    if (f) write(e, off + my);
    in_tile += round;
    __syncthreads();
  }
}

// rowptr_out[r] = number of kept entries before rowptr[r].
__global__ void k_rowptr_tiles(const int64_t* __restrict__ rowptr, int64_t n_rows, int64_t n,
                               const int64_t* __restrict__ tile_off,
                               const int32_t* __restrict__ pos_in_tile, int64_t n_tiles,
                               int64_t* __restrict__ rowptr_out) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (r > n_rows) return;
  const int64_t e0 = rowptr[r];
  rowptr_out[r] = e0 < n ? tile_off[e0 / kTile] + pos_in_tile[e0] : tile_off[n_tiles];
}

__global__ void k_copy_i64(const int64_t* __restrict__ src, int64_t* __restrict__ dst) {
  *dst = *src;
}

int64_t n_tiles_for(int64_t n) { return (n + kTile - 1) / kTile; }

size_t tile_ws_bytes(int64_t n, bool with_pos) {
  const int64_t t = n_tiles_for(n);
  return align_up(static_cast<size_t>(t + 1) * sizeof(int32_t)) +
         align_up(static_cast<size_t>(t + 1) * sizeof(int64_t)) +
         (with_pos ? align_up(static_cast<size_t>(n + 1) * sizeof(int32_t)) : 0);
}

// Launches count → scan → compact (+ optional in-tile positions) on `ws`.
template <class F, class W>
hgd_status tile_compact(F flag, W write, int64_t n, char* ws, bool with_pos, hipStream_t st,
                        int64_t** tile_off_out, int32_t** pos_out, const char* what) {
  const int64_t t = n_tiles_for(n);
  int32_t* cnt = reinterpret_cast<int32_t*>(ws);
  int64_t* off = reinterpret_cast<int64_t*>(ws + align_up(static_cast<size_t>(t + 1) * 4));
  int32_t* pos = with_pos ? reinterpret_cast<int32_t*>(
                                ws + align_up(static_cast<size_t>(t + 1) * 4) +
                                align_up(static_cast<size_t>(t + 1) * 8))
                          : nullptr;
  if (t > 0x7fffffffLL) return fail(HGD_ERR_UNSUPPORTED, "%s: too many tiles", what);
  hipLaunchKernelGGL((k_tile_count<F>), dim3(t), dim3(kTileThreads), 0, st, flag, n, cnt);
  hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(1024), 0, st, cnt, t, off);
  hipLaunchKernelGGL((k_tile_compact<F, W>), dim3(t), dim3(kTileThreads), 0, st, flag, write, n,
                     off, pos);
  *tile_off_out = off;
  if (pos_out) *pos_out = pos;
  return check_launch(what);
}

// Counter-based keep-mask: u = 24-bit uniform in [0,1) from a splitmix64 hash of (seed, i)
// (device_util.h); keep iff floor(u + keep) != 0, the expression of SpAdjDropEdge (HCCF.py:223)
// on a device RNG.

__global__ void k_bernoulli_mask(uint64_t seed, int64_t n, float keep,
                                 uint8_t* __restrict__ mask) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint64_t h = splitmix64(seed ^ splitmix64(static_cast<uint64_t>(i)));
  const float u = static_cast<float>(h >> 40) * (1.0f / 16777216.0f);
  mask[i] = floorf(u + keep) != 0.f ? 1 : 0;
}

// The same draw with the seed read from device memory (a counter a captured step advances).
__global__ void k_bernoulli_mask_dev(const uint64_t* __restrict__ seed_ptr, int64_t n, float keep,
                                     uint8_t* __restrict__ mask) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint64_t h = splitmix64(seed_ptr[0] ^ splitmix64(static_cast<uint64_t>(i)));
  const float u = static_cast<float>(h >> 40) * (1.0f / 16777216.0f);
  mask[i] = floorf(u + keep) != 0.f ? 1 : 0;
}

// Both orientations' masks of one device draw: mask[j] = bern(j) in CSR order and
// mask_t[j] = bern(perm_t[j]) in CSC order — the CSC mask without a random byte gather.
__device__ __forceinline__ uint8_t bern_bit(uint64_t seed, uint64_t i, float keep) {
  const uint64_t h = splitmix64(seed ^ splitmix64(i));
  const float u = static_cast<float>(h >> 40) * (1.0f / 16777216.0f);
  return floorf(u + keep) != 0.f ? 1 : 0;
}

__global__ void k_bernoulli_mask_dev_pair(const uint64_t* __restrict__ seed_ptr,
                                          const int32_t* __restrict__ perm_t, int64_t n,
                                          float keep, uint8_t* __restrict__ mask,
                                          uint8_t* __restrict__ mask_t) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint64_t seed = seed_ptr[0];
  mask[i] = bern_bit(seed, static_cast<uint64_t>(i), keep);
  mask_t[i] = bern_bit(seed, static_cast<uint64_t>(perm_t[i]), keep);
}

// Zeroes entries [*count, capacity) of a capacity-sized dropped structure (valid index 0,
// weight 0), so that nothing reading the arrays linearly meets uninitialised indices.
__global__ void k_fill_tail(const int64_t* __restrict__ count, int64_t capacity,
                            int32_t* __restrict__ col, float* __restrict__ val,
                            int32_t* __restrict__ row_t, float* __restrict__ val_t) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= capacity || i < count[0]) return;
  if (col) col[i] = 0;
  if (row_t) row_t[i] = 0;
  if (val) val[i] = 0.f;
  if (val_t) val_t[i] = 0.f;
}

// HGD_DENSE_GREATER: v > thresh (torch.nonzero(H > thresh)); HGD_DENSE_NONZERO: v != 0
// (torch.nonzero(H), the pattern of a dense adjacency such as DHCF's, DHCF.py:140).
__device__ __forceinline__ bool dense_keep(float v, float thresh, int mode) {
  return mode == HGD_DENSE_NONZERO ? v != 0.f : v > thresh;
}

// One wavefront per row: number of kept entries.
__global__ void k_dense_count(const float* __restrict__ H, int64_t n_rows, int64_t n_cols,
                              int64_t ld, float thresh, int mode,
                              int64_t* __restrict__ counts) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * (kBlock / 64) + threadIdx.x / 64;
  const int lane = threadIdx.x & 63;
  if (r > n_rows) return;
  int64_t cnt = 0;
  if (r < n_rows) {
    const float* row = H + r * ld;
    for (int64_t c0 = 0; c0 < n_cols; c0 += 64) {
      const int64_t c = c0 + lane;
      const bool f = c < n_cols && dense_keep(row[c], thresh, mode);
      cnt += __popcll(__ballot(f));
    }
  }
  if (lane == 0) counts[r] = cnt;  // counts[n_rows] = 0 → exclusive scan total
}

__global__ void k_dense_fill(const float* __restrict__ H, int64_t n_rows, int64_t n_cols,
                             int64_t ld, float thresh, int mode,
                             const int64_t* __restrict__ rowptr, int32_t* __restrict__ cols,
                             float* __restrict__ vals) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * (kBlock / 64) + threadIdx.x / 64;
  const int lane = threadIdx.x & 63;
  if (r >= n_rows) return;
  const float* row = H + r * ld;
  int64_t p = rowptr[r];
  const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int64_t c0 = 0; c0 < n_cols; c0 += 64) {
    const int64_t c = c0 + lane;
    const float v = c < n_cols ? row[c] : 0.f;
    const bool f = c < n_cols && dense_keep(v, thresh, mode);
    const unsigned long long b = __ballot(f);
    if (f) {
      const int64_t q = p + __popcll(b & lt_mask);
      cols[q] = static_cast<int32_t>(c);
      if (vals) vals[q] = v;
    }
    p += __popcll(b);
  }
}

template <typename T>
size_t excl_scan_bytes(int64_t n) {
  size_t bytes = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, static_cast<const T*>(nullptr),
                                       static_cast<T*>(nullptr), n) != hipSuccess)
    return 0;
  return bytes;
}

}  // namespace hgd

using namespace hgd;

extern "C" int hgd_version(void) { return 400; }  // 0.4.0

extern "C" const char* hgd_get_last_error_string(void) { return g_last_error; }

// ------------------------------------------------------------------------------------------
extern "C" hgd_status hgd_split_plan_count(const int64_t* rowptr, int64_t n_rows,
                                           int64_t threshold, int32_t chunk, int64_t* counts,
                                           void* stream) {
  clear_error();
  HGD_REQUIRE(rowptr && counts, "hgd_split_plan_count: null pointer");
  HGD_REQUIRE(chunk > 0 && threshold > 0, "hgd_split_plan_count: chunk/threshold must be > 0");
  hipStream_t st = as_stream(stream);
  HGD_HIP(hipMemsetAsync(counts, 0, 2 * sizeof(int64_t), st));
  if (n_rows <= 0) return HGD_OK;
  hipLaunchKernelGGL(k_plan_count, dim3(grid_for(n_rows)), dim3(kBlock), 0, st, rowptr, n_rows,
                     threshold, chunk, reinterpret_cast<unsigned long long*>(counts));
  return check_launch("hgd_split_plan_count");
}

extern "C" size_t hgd_split_plan_workspace_size(int64_t n_rows) {
  const size_t arr = align_up(static_cast<size_t>(n_rows + 1) * sizeof(int64_t));
  return 4 * arr + align_up(excl_scan_bytes<int64_t>(n_rows + 1));
}

extern "C" hgd_status hgd_split_plan_build(const int64_t* rowptr, int64_t n_rows,
                                           int64_t threshold, int32_t chunk, int32_t* heavy_rows,
                                           int64_t* heavy_cptr, int32_t* chunk_heavy,
                                           int64_t n_heavy, int64_t n_chunks, void* workspace,
                                           size_t workspace_bytes, void* stream) {
  clear_error();
  HGD_REQUIRE(rowptr && heavy_cptr, "hgd_split_plan_build: null pointer");
  HGD_REQUIRE(chunk > 0 && threshold > 0, "hgd_split_plan_build: chunk/threshold must be > 0");
  const size_t need = hgd_split_plan_workspace_size(n_rows);
  if (workspace_bytes < need || !workspace)
    return fail(HGD_ERR_WORKSPACE, "hgd_split_plan_build: workspace %zu < %zu", workspace_bytes,
                need);
  hipStream_t st = as_stream(stream);
  if (n_heavy == 0) {
    HGD_HIP(hipMemsetAsync(heavy_cptr, 0, sizeof(int64_t), st));
    return HGD_OK;
  }
  HGD_REQUIRE(heavy_rows && chunk_heavy, "hgd_split_plan_build: null output arrays");
  const size_t arr = align_up(static_cast<size_t>(n_rows + 1) * sizeof(int64_t));
  char* ws = static_cast<char*>(workspace);
  int64_t* flag = reinterpret_cast<int64_t*>(ws);
  int64_t* nch = reinterpret_cast<int64_t*>(ws + arr);
  int64_t* pos = reinterpret_cast<int64_t*>(ws + 2 * arr);
  int64_t* cpos = reinterpret_cast<int64_t*>(ws + 3 * arr);
  void* tmp = ws + 4 * arr;
  size_t tmp_bytes = workspace_bytes - 4 * arr;
  hipLaunchKernelGGL(k_plan_flags, dim3(grid_for(n_rows + 1)), dim3(kBlock), 0, st, rowptr,
                     n_rows, threshold, chunk, flag, nch);
  hgd_status s = check_launch("hgd_split_plan_build flags");
  if (s != HGD_OK) return s;
  size_t b = tmp_bytes;
  HGD_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, b, flag, pos, n_rows + 1, st));
  b = tmp_bytes;
  HGD_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, b, nch, cpos, n_rows + 1, st));
  hipLaunchKernelGGL(k_plan_scatter, dim3(grid_for(n_rows + 1)), dim3(kBlock), 0, st, rowptr,
                     n_rows, threshold, pos, cpos, heavy_rows, heavy_cptr, n_heavy);
  s = check_launch("hgd_split_plan_build scatter");
  if (s != HGD_OK) return s;
  if (n_chunks > 0) {
    hipLaunchKernelGGL(k_plan_chunks, dim3(grid_for(n_chunks)), dim3(kBlock), 0, st, heavy_cptr,
                       n_heavy, n_chunks, chunk_heavy);
    return check_launch("hgd_split_plan_build chunks");
  }
  return HGD_OK;
}

// ------------------------------------------------------------------------------------------
extern "C" hgd_status hgd_index_narrow(const int64_t* in, int64_t n, int64_t upper, int32_t* out,
                                       int64_t* err_count, void* stream) {
  clear_error();
  HGD_REQUIRE(n >= 0, "hgd_index_narrow: n < 0");
  HGD_REQUIRE(upper <= 0x7fffffffLL + 1, "hgd_index_narrow: upper bound exceeds int32");
  if (n == 0) return HGD_OK;
  HGD_REQUIRE(in && out && err_count, "hgd_index_narrow: null pointer");
  hipLaunchKernelGGL(k_index_narrow, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), in,
                     n, upper, out, reinterpret_cast<unsigned long long*>(err_count));
  return check_launch("hgd_index_narrow");
}

extern "C" size_t hgd_sort_perm_workspace_size(int64_t n) {
  size_t bytes = 0;
  if (n <= 0) return 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, static_cast<const int32_t*>(nullptr),
                                         static_cast<int32_t*>(nullptr),
                                         static_cast<const int32_t*>(nullptr),
                                         static_cast<int32_t*>(nullptr), n, 0, 32) != hipSuccess)
    return 0;
  return align_up(static_cast<size_t>(n) * sizeof(int32_t)) + align_up(bytes);
}

extern "C" hgd_status hgd_sort_perm(const int32_t* keys, int64_t n, int64_t n_keys,
                                    int32_t* keys_out, int32_t* perm_out, void* workspace,
                                    size_t workspace_bytes, void* stream) {
  clear_error();
  HGD_REQUIRE(n >= 0 && n < 0x7fffffffLL, "hgd_sort_perm: n out of range");
  if (n == 0) return HGD_OK;
  HGD_REQUIRE(keys && keys_out && perm_out, "hgd_sort_perm: null pointer");
  HGD_REQUIRE(n_keys > 0 && n_keys <= 0x7fffffffLL + 1, "hgd_sort_perm: bad n_keys");
  const size_t need = hgd_sort_perm_workspace_size(n);
  if (need == 0 || workspace_bytes < need || !workspace)
    return fail(HGD_ERR_WORKSPACE, "hgd_sort_perm: workspace %zu < %zu", workspace_bytes, need);
  hipStream_t st = as_stream(stream);
  char* ws = static_cast<char*>(workspace);
  int32_t* iota = reinterpret_cast<int32_t*>(ws);
  const size_t off = align_up(static_cast<size_t>(n) * sizeof(int32_t));
  hipLaunchKernelGGL(k_iota, dim3(grid_for(n)), dim3(kBlock), 0, st, iota, n);
  hgd_status s = check_launch("hgd_sort_perm iota");
  if (s != HGD_OK) return s;
  int end_bit = 1;
  while (end_bit < 32 && (1LL << end_bit) < n_keys) ++end_bit;
  size_t b = workspace_bytes - off;
  HGD_HIP(hipcub::DeviceRadixSort::SortPairs(ws + off, b, keys, keys_out, iota, perm_out, n, 0,
                                             end_bit, st));
  return HGD_OK;
}

extern "C" hgd_status hgd_rowptr_from_sorted(const int32_t* sorted_rows, int64_t nnz,
                                             int64_t n_rows, int64_t* rowptr, void* stream) {
  clear_error();
  HGD_REQUIRE(nnz >= 0 && n_rows >= 0, "hgd_rowptr_from_sorted: negative size");
  HGD_REQUIRE(rowptr && (sorted_rows || nnz == 0), "hgd_rowptr_from_sorted: null pointer");
  hipLaunchKernelGGL(k_rowptr_from_sorted, dim3(grid_for(n_rows + 1)), dim3(kBlock), 0,
                     as_stream(stream), sorted_rows, nnz, n_rows, rowptr);
  return check_launch("hgd_rowptr_from_sorted");
}

extern "C" hgd_status hgd_check_sorted(const int32_t* rows, int64_t nnz, int64_t n_rows,
                                       int64_t* bad, void* stream) {
  clear_error();
  HGD_REQUIRE(bad && (rows || nnz == 0), "hgd_check_sorted: null pointer");
  hipStream_t st = as_stream(stream);
  HGD_HIP(hipMemsetAsync(bad, 0, sizeof(int64_t), st));
  if (nnz == 0) return HGD_OK;
  hipLaunchKernelGGL(k_check_sorted, dim3(grid_for(nnz)), dim3(kBlock), 0, st, rows, nnz, n_rows,
                     reinterpret_cast<unsigned long long*>(bad));
  return check_launch("hgd_check_sorted");
}

extern "C" hgd_status hgd_expand_rows(const int64_t* rowptr, int64_t n_rows, int64_t nnz,
                                      int32_t* rows_out, void* stream) {
  clear_error();
  HGD_REQUIRE(rowptr && n_rows >= 0 && nnz >= 0, "hgd_expand_rows: bad arguments");
  if (nnz == 0) return HGD_OK;
  HGD_REQUIRE(rows_out && n_rows > 0, "hgd_expand_rows: null rows_out or no rows");
  hipLaunchKernelGGL(k_expand_rows, dim3(grid_for(nnz)), dim3(kBlock), 0, as_stream(stream),
                     rowptr, n_rows, rows_out, nnz);
  return check_launch("hgd_expand_rows");
}

extern "C" hgd_status hgd_gather32(const void* src, const int32_t* perm, int64_t n, void* out,
                                   void* stream) {
  clear_error();
  if (n == 0) return HGD_OK;
  HGD_REQUIRE(src && perm && out && n > 0, "hgd_gather32: bad arguments");
  hipLaunchKernelGGL(k_gather32, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream),
                     static_cast<const uint32_t*>(src), perm, n, static_cast<uint32_t*>(out));
  return check_launch("hgd_gather32");
}

extern "C" hgd_status hgd_gather_u8(const uint8_t* src, const int32_t* perm, int64_t n,
                                    uint8_t* out, void* stream) {
  clear_error();
  HGD_REQUIRE(n >= 0, "hgd_gather_u8: n < 0");
  if (n == 0) return HGD_OK;
  HGD_REQUIRE(src && perm && out, "hgd_gather_u8: null pointer");
  HGD_REQUIRE(reinterpret_cast<uintptr_t>(perm) % 16 == 0 && reinterpret_cast<uintptr_t>(out) % 4 == 0,
              "hgd_gather_u8: perm must be 16-byte and out 4-byte aligned");
  const int64_t threads = (n + 3) / 4;
  hipLaunchKernelGGL(k_gather_u8, dim3(grid_for(threads)), dim3(kBlock), 0, as_stream(stream),
                     src, perm, n, out);
  return check_launch("hgd_gather_u8");
}

extern "C" hgd_status hgd_degree_scale(const int64_t* rowptr, const float* val, int64_t n_rows,
                                       double power, float* scale_out, void* stream) {
  clear_error();
  HGD_REQUIRE(n_rows >= 0, "hgd_degree_scale: n_rows < 0");
  if (n_rows == 0) return HGD_OK;
  HGD_REQUIRE(rowptr && scale_out, "hgd_degree_scale: null pointer");
  hipLaunchKernelGGL(k_degree_scale, dim3(grid_for(n_rows)), dim3(kBlock), 0, as_stream(stream),
                     rowptr, val, n_rows, power, scale_out);
  return check_launch("hgd_degree_scale");
}

extern "C" hgd_status hgd_edge_values(const float* base, const int32_t* perm,
                                      const float* src_scale, const int32_t* src_idx, int64_t n,
                                      float* out, void* stream) {
  clear_error();
  HGD_REQUIRE(n >= 0, "hgd_edge_values: n < 0");
  if (n == 0) return HGD_OK;
  HGD_REQUIRE(out, "hgd_edge_values: null out");
  HGD_REQUIRE(!src_scale || src_idx, "hgd_edge_values: src_scale needs src_idx");
  HGD_REQUIRE(!perm || base, "hgd_edge_values: perm needs base");
  hipLaunchKernelGGL(k_edge_values, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), base,
                     perm, src_scale, src_idx, n, out);
  return check_launch("hgd_edge_values");
}

extern "C" size_t hgd_dropedge_workspace_size(int64_t nnz) {
  return tile_ws_bytes(nnz, false);
}

extern "C" hgd_status hgd_dropedge_compact(const int64_t* rows, const int64_t* cols,
                                           const float* val, const uint8_t* mask, int64_t nnz,
                                           float keep, int64_t* out_rows, int64_t* out_cols,
                                           float* out_val, int64_t* out_count, void* workspace,
                                           size_t workspace_bytes, void* stream) {
  clear_error();
  HGD_REQUIRE(nnz >= 0 && out_count, "hgd_dropedge_compact: bad arguments");
  HGD_REQUIRE(keep > 0.f, "hgd_dropedge_compact: keep must be > 0");
  hipStream_t st = as_stream(stream);
  if (nnz == 0) {
    HGD_HIP(hipMemsetAsync(out_count, 0, sizeof(int64_t), st));
    return HGD_OK;
  }
  HGD_REQUIRE(rows && cols && val && mask && out_rows && out_cols && out_val,
              "hgd_dropedge_compact: null pointer");
  const size_t need = hgd_dropedge_workspace_size(nnz);
  if (workspace_bytes < need || !workspace)
    return fail(HGD_ERR_WORKSPACE, "hgd_dropedge_compact: workspace %zu < %zu", workspace_bytes,
                need);
  int64_t* off = nullptr;
  hgd_status s = tile_compact(MaskFlag{mask, nullptr},
                              CooWriter{rows, cols, val, keep, out_rows, out_cols, out_val}, nnz,
                              static_cast<char*>(workspace), false, st, &off, nullptr,
                              "hgd_dropedge_compact");
  if (s != HGD_OK) return s;
  hipLaunchKernelGGL(k_copy_i64, dim3(1), dim3(1), 0, st, off + n_tiles_for(nnz), out_count);
  return check_launch("hgd_dropedge_compact count");
}

extern "C" hgd_status hgd_bernoulli_mask(uint64_t seed, int64_t n, float keep, uint8_t* mask,
                                         void* stream) {
  clear_error();
  HGD_REQUIRE(n >= 0 && (mask || n == 0), "hgd_bernoulli_mask: bad arguments");
  if (n == 0) return HGD_OK;
  hipLaunchKernelGGL(k_bernoulli_mask, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream),
                     seed, n, keep, mask);
  return check_launch("hgd_bernoulli_mask");
}

extern "C" hgd_status hgd_bernoulli_mask_dev(const uint64_t* seed, int64_t n, float keep,
                                             uint8_t* mask, void* stream) {
  clear_error();
  HGD_REQUIRE(n >= 0 && seed && (mask || n == 0), "hgd_bernoulli_mask_dev: bad arguments");
  if (n == 0) return HGD_OK;
  hipLaunchKernelGGL(k_bernoulli_mask_dev, dim3(grid_for(n)), dim3(kBlock), 0,
                     as_stream(stream), seed, n, keep, mask);
  return check_launch("hgd_bernoulli_mask_dev");
}

extern "C" hgd_status hgd_bernoulli_mask_dev_pair(const uint64_t* seed, const int32_t* perm_t,
                                                  int64_t n, float keep, uint8_t* mask,
                                                  uint8_t* mask_t, void* stream) {
  clear_error();
  HGD_REQUIRE(n >= 0 && seed && ((mask && mask_t && perm_t) || n == 0),
              "hgd_bernoulli_mask_dev_pair: bad arguments");
  if (n == 0) return HGD_OK;
  hipLaunchKernelGGL(k_bernoulli_mask_dev_pair, dim3(grid_for(n)), dim3(kBlock), 0,
                     as_stream(stream), seed, perm_t, n, keep, mask, mask_t);
  return check_launch("hgd_bernoulli_mask_dev_pair");
}

extern "C" hgd_status hgd_dropedge_fill_tail(const int64_t* count, int64_t capacity,
                                             int32_t* col, float* val, int32_t* row_t,
                                             float* val_t, void* stream) {
  clear_error();
  HGD_REQUIRE(capacity >= 0 && count, "hgd_dropedge_fill_tail: bad arguments");
  if (capacity == 0) return HGD_OK;
  hipLaunchKernelGGL(k_fill_tail, dim3(grid_for(capacity)), dim3(kBlock), 0, as_stream(stream),
                     count, capacity, col, val, row_t, val_t);
  return check_launch("hgd_dropedge_fill_tail");
}

extern "C" size_t hgd_dropedge_structure_workspace_size(int64_t nnz) {
  return tile_ws_bytes(nnz, true);
}

extern "C" hgd_status hgd_dropedge_structure(
    const int64_t* rowptr, const int32_t* col, const float* val, const int64_t* colptr,
    const int32_t* row_t, const float* val_t, const int32_t* perm_t, int64_t n_rows,
    int64_t n_cols, int64_t nnz, const uint8_t* mask, float keep, int64_t* rowptr_out,
    int32_t* col_out, float* val_out, int64_t* colptr_out, int32_t* row_t_out,
    float* val_t_out, void* workspace, size_t workspace_bytes, void* stream) {
  clear_error();
  HGD_REQUIRE(n_rows >= 0 && n_cols >= 0 && nnz >= 0, "hgd_dropedge_structure: sizes");
  HGD_REQUIRE(keep > 0.f, "hgd_dropedge_structure: keep must be > 0");
  HGD_REQUIRE(rowptr && colptr && rowptr_out && colptr_out, "hgd_dropedge_structure: null ptr");
  HGD_REQUIRE(nnz == 0 || (col && row_t && perm_t && mask && col_out && row_t_out),
              "hgd_dropedge_structure: null index arrays");
  HGD_REQUIRE(!val == !val_t && (!val || (val_out && val_t_out)),
              "hgd_dropedge_structure: values must be given for both orientations or neither");
  const size_t need = hgd_dropedge_structure_workspace_size(nnz);
  if (workspace_bytes < need || !workspace)
    return fail(HGD_ERR_WORKSPACE, "hgd_dropedge_structure: workspace %zu < %zu",
                workspace_bytes, need);
  hipStream_t st = as_stream(stream);
  const int64_t nt = n_tiles_for(nnz);
  // the two orientations run one after the other on the same workspace (stream-ordered)
  for (int side = 0; side < 2; ++side) {
    const bool csc = side == 1;
    const int64_t nr = csc ? n_cols : n_rows;
    const int64_t* ptr = csc ? colptr : rowptr;
    int64_t* ptr_out = csc ? colptr_out : rowptr_out;
    int64_t* off = nullptr;
    int32_t* pos = nullptr;
    if (nnz > 0) {
      // CSR: the mask is in CSR order; CSC: entry e is CSR entry perm_t[e]
      hgd_status s = tile_compact(
          MaskFlag{mask, csc ? perm_t : nullptr},
          StructWriter{csc ? row_t : col, csc ? val_t : val, keep, csc ? row_t_out : col_out,
                       csc ? val_t_out : val_out},
          nnz, static_cast<char*>(workspace), true, st, &off, &pos,
          "hgd_dropedge_structure compact");
      if (s != HGD_OK) return s;
      hipLaunchKernelGGL(k_rowptr_tiles, dim3(grid_for(nr + 1)), dim3(kBlock), 0, st, ptr, nr,
                         nnz, off, pos, nt, ptr_out);
      s = check_launch("hgd_dropedge_structure rowptr");
      if (s != HGD_OK) return s;
    } else {
      HGD_HIP(hipMemsetAsync(ptr_out, 0, static_cast<size_t>(nr + 1) * sizeof(int64_t), st));
    }
  }
  return HGD_OK;
}

extern "C" size_t hgd_dense_threshold_workspace_size(int64_t n_rows) {
  return align_up(static_cast<size_t>(n_rows + 1) * sizeof(int64_t)) +
         align_up(excl_scan_bytes<int64_t>(n_rows + 1));
}

extern "C" hgd_status hgd_dense_threshold_rowptr(const float* H, int64_t n_rows, int64_t n_cols,
                                                 int64_t ld, float thresh, int32_t mode,
                                                 int64_t* rowptr, void* workspace,
                                                 size_t workspace_bytes, void* stream) {
  clear_error();
  HGD_REQUIRE(n_rows >= 0 && n_cols >= 0 && (ld >= n_cols || n_rows == 0),
              "hgd_dense_threshold_rowptr: sizes");
  HGD_REQUIRE(mode == HGD_DENSE_GREATER || mode == HGD_DENSE_NONZERO,
              "hgd_dense_threshold_rowptr: bad mode %d", mode);
  HGD_REQUIRE(rowptr && (H || n_rows == 0 || n_cols == 0), "hgd_dense_threshold_rowptr: null");
  const size_t need = hgd_dense_threshold_workspace_size(n_rows);
  if (workspace_bytes < need || !workspace)
    return fail(HGD_ERR_WORKSPACE, "hgd_dense_threshold_rowptr: workspace %zu < %zu",
                workspace_bytes, need);
  hipStream_t st = as_stream(stream);
  const size_t arr = align_up(static_cast<size_t>(n_rows + 1) * sizeof(int64_t));
  char* ws = static_cast<char*>(workspace);
  int64_t* counts = reinterpret_cast<int64_t*>(ws);
  hipLaunchKernelGGL(k_dense_count, dim3(grid_for(n_rows + 1, kBlock / 64)), dim3(kBlock), 0, st,
                     H, n_rows, n_cols, ld, thresh, mode, counts);
  hgd_status s = check_launch("hgd_dense_threshold_rowptr count");
  if (s != HGD_OK) return s;
  size_t b = workspace_bytes - arr;
  HGD_HIP(hipcub::DeviceScan::ExclusiveSum(ws + arr, b, counts, rowptr, n_rows + 1, st));
  return HGD_OK;
}

extern "C" hgd_status hgd_dense_threshold_fill(const float* H, int64_t n_rows, int64_t n_cols,
                                               int64_t ld, float thresh, int32_t mode,
                                               const int64_t* rowptr, int32_t* cols, float* vals,
                                               void* stream) {
  clear_error();
  HGD_REQUIRE(n_rows >= 0 && n_cols >= 0 && (ld >= n_cols || n_rows == 0),
              "hgd_dense_threshold_fill: sizes");
  HGD_REQUIRE(mode == HGD_DENSE_GREATER || mode == HGD_DENSE_NONZERO,
              "hgd_dense_threshold_fill: bad mode %d", mode);
  if (n_rows == 0 || n_cols == 0) return HGD_OK;
  HGD_REQUIRE(H && rowptr && cols, "hgd_dense_threshold_fill: null pointer");
  hipLaunchKernelGGL(k_dense_fill, dim3(grid_for(n_rows, kBlock / 64)), dim3(kBlock), 0,
                     as_stream(stream), H, n_rows, n_cols, ld, thresh, mode, rowptr, cols, vals);
  return check_launch("hgd_dense_threshold_fill");
}
