// Sorted unique of integer keys: torch.unique(x.long()) as HCCF's loss calls it on every step,
// `contrastLoss(..., torch.unique(ancs.long()), ...)` (model/graph/HCCF.py:65-66), over a
// [batch, d] float embedding block (262,144 values at batch 4096, d = 64). torch runs a device
// merge sort for it — ~20 launches per call, ~0.7 ms of an HCCF step (profiles/r01_hccf) —
// although the truncated values span a handful of integers.
//
// Here: a range bitmap. One pass finds min / max; if the range fits kCapBits, every key sets its
// bit (block-private LDS bitmap first when the range is small, so the hot words see one global
// atomicOr per block — OR is idempotent, so the result does not depend on the order), then a
// tile count / one-block scan / emit pass writes the set bits in ascending order: exactly
// torch.unique's sorted output. No host synchronisation: a range beyond the bitmap writes
// *n_out = -1 and the caller runs hgd_unique_sort (radix sort + unique, same result).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <climits>

#include "device_util.h"
#include "hgd_internal.h"

namespace hgd {
namespace {

constexpr int64_t kCapBits = int64_t(1) << 24;  // 2 MB bitmap
constexpr int64_t kCapWords = kCapBits / 32;
constexpr int kEmitThreads = 256;
constexpr int kWordsPerThread = 8;
constexpr int64_t kTileWords = kEmitThreads * kWordsPerThread;  // 2048 words = 65,536 bits
constexpr int64_t kMaxTiles = kCapWords / kTileWords;           // 256
constexpr int kLdsWords = 1024;                                 // block-private bitmap
constexpr unsigned kGrid = 512;

struct State {
  long long lo, hi;  // min / max key
  int overflow;
  int pad;
  unsigned long long far_n;  // device-complete path: keys beyond the bitmap window
};

struct I64Src {
  const int64_t* p;
  __device__ int64_t operator()(int64_t i) const { return p[i]; }
};

// float → int64 like Tensor.long(): truncation toward zero; NaN / ±inf / |x| >= 2^63 (undefined
// in C++) map to INT64_MIN, the x86 "integer indefinite" torch's CPU cast produces.
struct TruncSrc {
  const float* p;
  __device__ int64_t operator()(int64_t i) const {
    const float x = p[i];
    if (!(fabsf(x) < 9.2233720368547758e18f)) return INT64_MIN;
    return static_cast<int64_t>(x);
  }
};

__device__ __forceinline__ long long wave_min(long long v) {
  for (int o = 32; o > 0; o >>= 1) {
    const long long w = __shfl_xor(v, o);
    v = w < v ? w : v;
  }
  return v;
}
__device__ __forceinline__ long long wave_max(long long v) {
  for (int o = 32; o > 0; o >>= 1) {
    const long long w = __shfl_xor(v, o);
    v = w > v ? w : v;
  }
  return v;
}

__device__ __forceinline__ void uq_init(State* st) {
  st->lo = LLONG_MAX;
  st->hi = LLONG_MIN;
  st->overflow = 0;
  st->far_n = 0;
}

template <class Src>
__device__ __forceinline__ void uq_minmax(Src src, int64_t n, State* st) {
  long long lo = LLONG_MAX, hi = LLONG_MIN;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += stride) {
    const long long k = src(i);
    lo = k < lo ? k : lo;
    hi = k > hi ? k : hi;
  }
  lo = wave_min(lo);
  hi = wave_max(hi);
  // one atomic pair per workgroup: every wave hitting the same two words serialised them
  __shared__ long long s_lo[4], s_hi[4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_lo[w] = lo;
    s_hi[w] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 4; ++i) {
      lo = s_lo[i] < lo ? s_lo[i] : lo;
      hi = s_hi[i] > hi ? s_hi[i] : hi;
    }
    if (lo <= hi) {
      atomicMin(&st->lo, lo);
      atomicMax(&st->hi, hi);
    }
  }
}

// Bitmap words of the key range. CLAMP (the device-complete path): a range beyond the bitmap
// keeps the window [lo, lo + kCapBits) and the keys past it go to the far-key list instead.
template <bool CLAMP = false>
__device__ __forceinline__ bool range_words(const State* st, int64_t* words) {
  const long long lo = st->lo, hi = st->hi;
  if (lo > hi) {  // no keys
    *words = 0;
    return true;
  }
  // hi - lo may overflow int64: compare in unsigned
  unsigned long long span = static_cast<unsigned long long>(hi) -
                            static_cast<unsigned long long>(lo);
  if (span >= static_cast<unsigned long long>(kCapBits)) {
    if (!CLAMP) return false;
    span = static_cast<unsigned long long>(kCapBits) - 1;
  }
  *words = static_cast<int64_t>((span + 1 + 31) / 32);
  return true;
}

template <bool CLAMP>
__device__ __forceinline__ void uq_zero(uint32_t* bitmap, State* st) {
  int64_t words;
  if (!range_words<CLAMP>(st, &words)) {
    if (blockIdx.x == 0 && threadIdx.x == 0) st->overflow = 1;
    return;
  }
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t w = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; w < words;
       w += stride)
    bitmap[w] = 0u;
}

// Sets every key's bit. FAR (device-complete path): keys past the kCapBits window are appended
// to `far` (State::far_n counts them) instead.
template <class Src, bool FAR = false>
__device__ __forceinline__ void uq_mark(Src src, int64_t n, uint32_t* bitmap, State* st,
                                        int64_t* far) {
  __shared__ uint32_t s_bits[kLdsWords];
  int64_t words;
  if (!range_words<FAR>(st, &words) || words == 0) return;  // uniform over the grid
  const long long lo = st->lo;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const int64_t i0 = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  auto far_key = [&](uint64_t b, int64_t key) {
    if constexpr (FAR) {
      if (b >= static_cast<uint64_t>(kCapBits)) {
        const unsigned long long p = atomicAdd(&st->far_n, 1ull);
        far[p] = key;
        return true;
      }
    }
    return false;
  };
  if (words <= kLdsWords) {
    for (int w = threadIdx.x; w < words; w += blockDim.x) s_bits[w] = 0u;
    __syncthreads();
    for (int64_t i = i0; i < n; i += stride) {
      const int64_t key = src(i);
      const uint64_t b = static_cast<uint64_t>(key) - static_cast<uint64_t>(lo);
      if (!far_key(b, key)) atomicOr(&s_bits[b >> 5], 1u << (b & 31));
    }
    __syncthreads();
    for (int w = threadIdx.x; w < words; w += blockDim.x)
      if (s_bits[w]) atomicOr(&bitmap[w], s_bits[w]);
  } else {
    for (int64_t i = i0; i < n; i += stride) {
      const int64_t key = src(i);
      const uint64_t b = static_cast<uint64_t>(key) - static_cast<uint64_t>(lo);
      if (!far_key(b, key)) atomicOr(&bitmap[b >> 5], 1u << (b & 31));
    }
  }
}

__device__ __forceinline__ int block_exclusive_scan(int v, int* total) {
  __shared__ int s_wave[kEmitThreads / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int incl = v;
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(incl, o);
    if (lane >= o) incl += u;
  }
  if (lane == 63) s_wave[wave] = incl;
  __syncthreads();
  int base = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kEmitThreads / 64; ++w) {
    base += w < wave ? s_wave[w] : 0;
    all += s_wave[w];
  }
  *total = all;
  return base + incl - v;
}

template <bool CLAMP>
__device__ __forceinline__ void uq_count(const uint32_t* bitmap, const State* st,
                                         int* tile_cnt) {
  int64_t words;
  if (!range_words<CLAMP>(st, &words)) return;
  const int64_t tiles = (words + kTileWords - 1) / kTileWords;
  if (blockIdx.x >= tiles) return;
  const int64_t w0 = blockIdx.x * kTileWords + threadIdx.x * kWordsPerThread;
  int c = 0;
#pragma unroll
  for (int j = 0; j < kWordsPerThread; ++j)
    if (w0 + j < words) c += __popc(bitmap[w0 + j]);
  int total;
  (void)block_exclusive_scan(c, &total);
  if (threadIdx.x == 0) tile_cnt[blockIdx.x] = total;
}

template <bool CLAMP>
__device__ __forceinline__ void uq_scan(const int* tile_cnt, const State* st, int64_t* tile_off,
                                        int64_t* n_out) {
  __shared__ int64_t s[kMaxTiles];
  int64_t words;
  if (!range_words<CLAMP>(st, &words)) {
    if (threadIdx.x == 0) *n_out = -1;  // the caller runs hgd_unique_sort
    return;
  }
  const int64_t tiles = (words + kTileWords - 1) / kTileWords;
  const int64_t v = threadIdx.x < tiles ? tile_cnt[threadIdx.x] : 0;
  s[threadIdx.x] = v;
  __syncthreads();
  for (int d = 1; d < kMaxTiles; d <<= 1) {
    const int64_t u = static_cast<int>(threadIdx.x) >= d ? s[threadIdx.x - d] : 0;
    __syncthreads();
    s[threadIdx.x] += u;
    __syncthreads();
  }
  if (threadIdx.x < tiles) tile_off[threadIdx.x] = s[threadIdx.x] - v;
  if (threadIdx.x == kMaxTiles - 1) *n_out = s[threadIdx.x];
}

template <bool CLAMP>
__device__ __forceinline__ void uq_emit(const uint32_t* bitmap, const State* st,
                                        const int64_t* tile_off, int64_t* out) {
  int64_t words;
  if (!range_words<CLAMP>(st, &words)) return;
  const int64_t tiles = (words + kTileWords - 1) / kTileWords;
  if (blockIdx.x >= tiles) return;
  const long long lo = st->lo;
  const int64_t w0 = blockIdx.x * kTileWords + threadIdx.x * kWordsPerThread;
  uint32_t bits[kWordsPerThread];
  int c = 0;
#pragma unroll
  for (int j = 0; j < kWordsPerThread; ++j) {
    bits[j] = w0 + j < words ? bitmap[w0 + j] : 0u;
    c += __popc(bits[j]);
  }
  int total;
  int64_t pos = tile_off[blockIdx.x] + block_exclusive_scan(c, &total);
#pragma unroll
  for (int j = 0; j < kWordsPerThread; ++j) {
    uint32_t b = bits[j];
    while (b) {
      const int k = __ffs(b) - 1;
      b &= b - 1;
      out[pos++] = static_cast<int64_t>(static_cast<unsigned long long>(lo) +
                                        static_cast<unsigned long long>((w0 + j) * 32 + k));
    }
  }
}

// The far keys (device-complete path), one workgroup: nothing to do in the common case (every
// key inside the bitmap window: one load and exit). Otherwise they are sorted — in LDS when they
// fit kFarLds, else by an in-place bitonic network over the workspace (P = next power of two;
// slow but bounded: a degenerate input such as a NaN embedding, whose INT64_MIN key drags the
// window away from the others) — and their distinct values appended after the bitmap's, which
// are all smaller: the output stays torch.unique's sorted order.
constexpr int kFarThreads = 1024;
constexpr int kFarLds = 4096;

__device__ __forceinline__ void cas(int64_t& a, int64_t& b, bool up) {
  if ((a > b) == up) {
    const int64_t t = a;
    a = b;
    b = t;
  }
}

// Bitonic sort of keys[0, P) (P a power of two) by one workgroup; KEYS is the LDS array or the
// workspace buffer, indexed directly (no pointer that may be either).
template <class Keys>
__device__ __forceinline__ void block_bitonic(Keys& keys, int P) {
  const int t = threadIdx.x;
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = t; i < P / 2; i += kFarThreads) {
        const int lo_i = 2 * i - (i & (stride - 1));
        const bool up = (lo_i & size) == 0;
        int64_t x = keys[lo_i], y = keys[lo_i + stride];
        cas(x, y, up);
        keys[lo_i] = x;
        keys[lo_i + stride] = y;
      }
      __syncthreads();
    }
  }
}

__device__ __forceinline__ void uq_far(State* st, int64_t* far, int64_t cap, int64_t* out,
                                       int64_t* n_out, int64_t n) {
  __shared__ int64_t s_keys[kFarLds];
  __shared__ int s_wave[kFarThreads / 64];
  int64_t kk = static_cast<int64_t>(st->far_n);
  if (kk == 0) return;  // uniform
  kk = kk < cap ? kk : cap;  // defensive: never past the far buffer
  const int k = static_cast<int>(kk);
  const int t = threadIdx.x;
  int P = 1;
  while (P < k) P <<= 1;
  const bool lds = P <= kFarLds;
  if (lds) {
    for (int i = t; i < P; i += kFarThreads) s_keys[i] = i < k ? far[i] : LLONG_MAX;
    __syncthreads();
    block_bitonic(s_keys, P);
  } else {
    for (int i = k + t; i < P; i += kFarThreads) far[i] = LLONG_MAX;
    __syncthreads();
    block_bitonic(far, P);
  }
  // distinct values of the sorted first k, in chunks of kFarThreads with a running offset
  int64_t base = *n_out;
  for (int c0 = 0; c0 < k; c0 += kFarThreads) {
    const int i = c0 + t;
    int f = 0;
    int64_t v = 0;
    if (i < k) {
      v = lds ? s_keys[i] : far[i];
      const int64_t prev = i == 0 ? 0 : (lds ? s_keys[i - 1] : far[i - 1]);
      f = (i == 0 || v != prev) ? 1 : 0;
    }
    const int lane = t & 63, wave = t >> 6;
    int incl = f;
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(incl, o);
      if (lane >= o) incl += u;
    }
    if (lane == 63) s_wave[wave] = incl;
    __syncthreads();
    int pre = 0, tot = 0;
    for (int w = 0; w < kFarThreads / 64; ++w) {
      pre += w < wave ? s_wave[w] : 0;
      tot += s_wave[w];
    }
    const int64_t pos = base + pre + incl - f;
    if (f && pos >= 0 && pos < n) out[pos] = v;  // bounds: defensive, never false for valid state
    base += tot;
    __syncthreads();
  }
  if (t == 0) *n_out = base;
}

// Single-call kernels (the bodies above) and the grouped forms of the device-complete path
// (hgd_unique_dev_group: blockIdx.y picks the call, so several node lists share each launch).
__global__ void k_uq_init(State* st) { uq_init(st); }
template <class Src>
__global__ __launch_bounds__(256) void k_uq_minmax(Src src, int64_t n, State* st) {
  uq_minmax(src, n, st);
}
template <bool CLAMP>
__global__ __launch_bounds__(256) void k_uq_zero(uint32_t* bitmap, State* st) {
  uq_zero<CLAMP>(bitmap, st);
}
template <class Src, bool FAR = false>
__global__ __launch_bounds__(256) void k_uq_mark(Src src, int64_t n, uint32_t* bitmap, State* st,
                                                 int64_t* far = nullptr) {
  uq_mark<Src, FAR>(src, n, bitmap, st, far);
}
template <bool CLAMP>
__global__ __launch_bounds__(kEmitThreads) void k_uq_count(const uint32_t* bitmap, const State* st,
                                                           int* tile_cnt) {
  uq_count<CLAMP>(bitmap, st, tile_cnt);
}
template <bool CLAMP>
__global__ __launch_bounds__(kMaxTiles) void k_uq_scan(const int* tile_cnt, const State* st,
                                                       int64_t* tile_off, int64_t* n_out) {
  uq_scan<CLAMP>(tile_cnt, st, tile_off, n_out);
}
template <bool CLAMP>
__global__ __launch_bounds__(kEmitThreads) void k_uq_emit(const uint32_t* bitmap, const State* st,
                                                          const int64_t* tile_off, int64_t* out) {
  uq_emit<CLAMP>(bitmap, st, tile_off, out);
}
__global__ __launch_bounds__(kFarThreads) void k_uq_far(State* st, int64_t* far, int64_t cap,
                                                        int64_t* out, int64_t* n_out, int64_t n) {
  uq_far(st, far, cap, out, n_out, n);
}

// A key source of either type (a group may mix float and int64 lists).
struct AnySrc {
  const float* f;
  const int64_t* i;
  __device__ int64_t operator()(int64_t k) const {
    return f ? TruncSrc{f}(k) : i[k];
  }
};

constexpr int kMaxJobs = 4;
struct UqJob {
  AnySrc src;
  int64_t n;
  int64_t* out;
  int64_t* n_out;
  State* st;
  int* cnt;
  int64_t* toff;
  uint32_t* bitmap;
  int64_t* far;
  int64_t far_cap;
  int64_t cap;  // entries kept: n_out clamped to it, out[n_out, cap) zeroed
};
struct UqJobs {
  UqJob j[kMaxJobs];
};

__global__ void k_uqg_init(UqJobs J) { uq_init(J.j[blockIdx.y].st); }
__global__ __launch_bounds__(256) void k_uqg_minmax(UqJobs J) {
  const UqJob& j = J.j[blockIdx.y];
  uq_minmax(j.src, j.n, j.st);
}
__global__ __launch_bounds__(256) void k_uqg_zero(UqJobs J) {
  const UqJob& j = J.j[blockIdx.y];
  uq_zero<true>(j.bitmap, j.st);
}
__global__ __launch_bounds__(256) void k_uqg_mark(UqJobs J) {
  const UqJob& j = J.j[blockIdx.y];
  uq_mark<AnySrc, true>(j.src, j.n, j.bitmap, j.st, j.far);
}
__global__ __launch_bounds__(kEmitThreads) void k_uqg_count(UqJobs J) {
  const UqJob& j = J.j[blockIdx.y];
  uq_count<true>(j.bitmap, j.st, j.cnt);
}
__global__ __launch_bounds__(kMaxTiles) void k_uqg_scan(UqJobs J) {
  const UqJob& j = J.j[blockIdx.y];
  uq_scan<true>(j.cnt, j.st, j.toff, j.n_out);
}
__global__ __launch_bounds__(kEmitThreads) void k_uqg_emit(UqJobs J) {
  const UqJob& j = J.j[blockIdx.y];
  uq_emit<true>(j.bitmap, j.st, j.toff, j.out);
}
__global__ __launch_bounds__(kFarThreads) void k_uqg_far(UqJobs J) {
  const UqJob& j = J.j[blockIdx.y];
  uq_far(j.st, j.far, j.far_cap, j.out, j.n_out, j.n);
}
// n_out = min(n_out, cap) and out[n_out, cap) = 0. Every block derives the same clamped count
// (min is idempotent, so reading before or after block 0's store gives the same value).
__global__ __launch_bounds__(256) void k_uqg_tail(UqJobs J) {
  const UqJob& j = J.j[blockIdx.y];
  const int64_t raw = *j.n_out;
  const int64_t c = raw < j.cap ? raw : j.cap;
  for (int64_t i = c + blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < j.cap;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    j.out[i] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0 && raw > j.cap) *j.n_out = j.cap;
}

template <class Src>
__global__ void k_uq_materialize(Src src, int64_t n, int64_t* keys) {
  const int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (i < n) keys[i] = src(i);
}

// workspace layout of the bitmap path
constexpr size_t kOffState = 0;
constexpr size_t kOffCnt = 256;
constexpr size_t kOffTileOff = kOffCnt + kMaxTiles * sizeof(int);
constexpr size_t kOffBitmap = kOffTileOff + kMaxTiles * sizeof(int64_t);
constexpr size_t kBitmapPathBytes = kOffBitmap + kCapWords * sizeof(uint32_t);

size_t sort_path_bytes(int64_t n) {
  size_t a = 0, b = 0;
  if (hipcub::DeviceRadixSort::SortKeys(nullptr, a, static_cast<const int64_t*>(nullptr),
                                        static_cast<int64_t*>(nullptr), static_cast<int>(n)) !=
      hipSuccess)
    return 0;
  if (hipcub::DeviceSelect::Unique(nullptr, b, static_cast<const int64_t*>(nullptr),
                                   static_cast<int64_t*>(nullptr), static_cast<int64_t*>(nullptr),
                                   static_cast<int>(n)) != hipSuccess)
    return 0;
  return 2 * align_up(static_cast<size_t>(n) * 8) + align_up(a > b ? a : b);
}

int64_t far_capacity(int64_t n) {
  int64_t p = 1;
  while (p < n) p <<= 1;
  return p;
}

size_t dev_path_bytes(int64_t n) {
  return kBitmapPathBytes + align_up(static_cast<size_t>(far_capacity(n)) * 8);
}

// DEV (device-complete): the window clamps instead of failing and the far keys are merged by
// k_uq_far, so *n_out is always the unique count — no host decision, capturable in a graph.
template <class Src, bool DEV = false>
hgd_status unique_bitmap(Src src, int64_t n, int64_t* out, int64_t* n_out, void* ws, size_t wsb,
                         hipStream_t st, const char* fn) {
  HGD_REQUIRE(n >= 0 && n < (int64_t(1) << 31), "%s: n must be in [0, 2^31)", fn);
  HGD_REQUIRE(n_out && (n == 0 || out), "%s: null output", fn);
  const size_t need = DEV ? dev_path_bytes(n) : kBitmapPathBytes;
  if (wsb < need || !ws)
    return fail(HGD_ERR_WORKSPACE, "%s: workspace %zu < required %zu", fn, wsb, need);
  char* w = static_cast<char*>(ws);
  int64_t* far = DEV ? reinterpret_cast<int64_t*>(w + kBitmapPathBytes) : nullptr;
  const int64_t far_cap = DEV ? far_capacity(n) : 0;
  State* s = reinterpret_cast<State*>(w + kOffState);
  int* cnt = reinterpret_cast<int*>(w + kOffCnt);
  int64_t* toff = reinterpret_cast<int64_t*>(w + kOffTileOff);
  uint32_t* bitmap = reinterpret_cast<uint32_t*>(w + kOffBitmap);
  hipLaunchKernelGGL(k_uq_init, dim3(1), dim3(1), 0, st, s);
  if (n > 0) {  // >= 16 keys per thread before the workgroup's atomic pair
    const unsigned g = static_cast<unsigned>(std::min<int64_t>(kGrid, (n + 4095) / 4096));
    hipLaunchKernelGGL(k_uq_minmax<Src>, dim3(g), dim3(256), 0, st, src, n, s);
  }
  hipLaunchKernelGGL(k_uq_zero<DEV>, dim3(kGrid), dim3(256), 0, st, bitmap, s);
  if (n > 0) {
    const unsigned g = static_cast<unsigned>(std::min<int64_t>(kGrid, (n + 255) / 256));
    hipLaunchKernelGGL((k_uq_mark<Src, DEV>), dim3(g), dim3(256), 0, st, src, n, bitmap, s, far);
  }
  hipLaunchKernelGGL(k_uq_count<DEV>, dim3(kMaxTiles), dim3(kEmitThreads), 0, st, bitmap, s, cnt);
  hipLaunchKernelGGL(k_uq_scan<DEV>, dim3(1), dim3(kMaxTiles), 0, st, cnt, s, toff, n_out);
  hipLaunchKernelGGL(k_uq_emit<DEV>, dim3(kMaxTiles), dim3(kEmitThreads), 0, st, bitmap, s, toff,
                     out);
  if (DEV) hipLaunchKernelGGL(k_uq_far, dim3(1), dim3(kFarThreads), 0, st, s, far, far_cap, out,
                              n_out, n);
  return check_launch(fn);
}

template <class Src>
hgd_status unique_sort(Src src, const int64_t* keys_in, int64_t n, int64_t* out, int64_t* n_out,
                       void* ws, size_t wsb, hipStream_t st, const char* fn) {
  HGD_REQUIRE(n >= 0 && n < (int64_t(1) << 31), "%s: n must be in [0, 2^31)", fn);
  HGD_REQUIRE(n_out && (n == 0 || out), "%s: null output", fn);
  if (n == 0) {
    HGD_HIP(hipMemsetAsync(n_out, 0, sizeof(int64_t), st));
    return HGD_OK;
  }
  const size_t need = sort_path_bytes(n);
  if (need == 0) return fail(HGD_ERR_HIP, "%s: hipcub workspace query failed", fn);
  if (wsb < need || !ws)
    return fail(HGD_ERR_WORKSPACE, "%s: workspace %zu < required %zu", fn, wsb, need);
  char* w = static_cast<char*>(ws);
  int64_t* keys = reinterpret_cast<int64_t*>(w);
  int64_t* sorted = reinterpret_cast<int64_t*>(w + align_up(static_cast<size_t>(n) * 8));
  char* tmp = w + 2 * align_up(static_cast<size_t>(n) * 8);
  size_t tb = wsb - 2 * align_up(static_cast<size_t>(n) * 8);
  if (!keys_in) {
    hipLaunchKernelGGL(k_uq_materialize<Src>, dim3(grid_for(n)), dim3(kBlock), 0, st, src, n,
                       keys);
    hgd_status r = check_launch(fn);
    if (r != HGD_OK) return r;
    keys_in = keys;
  }
  HGD_HIP(hipcub::DeviceRadixSort::SortKeys(tmp, tb, keys_in, sorted, static_cast<int>(n), 0, 64,
                                            st));
  HGD_HIP(hipcub::DeviceSelect::Unique(tmp, tb, sorted, out, n_out, static_cast<int>(n), st));
  return HGD_OK;
}

// The device-complete path for several lists at once: the same kernels, one launch each for
// all of them (grid y = the list), every list exactly as hgd_unique_dev_* would give it.
hgd_status unique_group(const hgd_unique_job* jobs, int count, hipStream_t st, const char* fn) {
  HGD_REQUIRE(jobs && count >= 1 && count <= kMaxJobs, "%s: 1 to %d lists", fn, kMaxJobs);
  UqJobs J{};
  int64_t n_max = 0;
  for (int k = 0; k < count; ++k) {
    const hgd_unique_job& q = jobs[k];
    HGD_REQUIRE(q.n >= 0 && q.n < (int64_t(1) << 31), "%s: list %d: n must be in [0, 2^31)", fn, k);
    HGD_REQUIRE(q.n_out && (q.n == 0 || q.out), "%s: list %d: null output", fn, k);
    HGD_REQUIRE(q.n == 0 || (q.x_f32 != nullptr) != (q.x_i64 != nullptr),
                "%s: list %d: exactly one of x_f32 / x_i64", fn, k);
    const size_t need = dev_path_bytes(q.n);
    if (q.workspace_bytes < need || !q.workspace)
      return fail(HGD_ERR_WORKSPACE, "%s: list %d: workspace %zu < required %zu", fn, k,
                  q.workspace_bytes, need);
    char* w = static_cast<char*>(q.workspace);
    UqJob& j = J.j[k];
    j.src = AnySrc{q.x_f32, q.x_i64};
    j.n = q.n;
    j.out = q.out;
    j.n_out = q.n_out;
    j.st = reinterpret_cast<State*>(w + kOffState);
    j.cnt = reinterpret_cast<int*>(w + kOffCnt);
    j.toff = reinterpret_cast<int64_t*>(w + kOffTileOff);
    j.bitmap = reinterpret_cast<uint32_t*>(w + kOffBitmap);
    j.far = reinterpret_cast<int64_t*>(w + kBitmapPathBytes);
    j.far_cap = far_capacity(q.n);
    HGD_REQUIRE(q.capacity >= 0 && q.capacity <= q.n, "%s: list %d: capacity must be in [0, n]",
                fn, k);
    j.cap = q.capacity > 0 ? q.capacity : q.n;
    n_max = std::max(n_max, q.n);
  }
  const unsigned y = static_cast<unsigned>(count);
  hipLaunchKernelGGL(k_uqg_init, dim3(1, y), dim3(1), 0, st, J);
  if (n_max > 0) {
    const unsigned g = static_cast<unsigned>(std::min<int64_t>(kGrid, (n_max + 4095) / 4096));
    hipLaunchKernelGGL(k_uqg_minmax, dim3(g, y), dim3(256), 0, st, J);
  }
  hipLaunchKernelGGL(k_uqg_zero, dim3(kGrid, y), dim3(256), 0, st, J);
  if (n_max > 0) {
    const unsigned g = static_cast<unsigned>(std::min<int64_t>(kGrid, (n_max + 255) / 256));
    hipLaunchKernelGGL(k_uqg_mark, dim3(g, y), dim3(256), 0, st, J);
  }
  hipLaunchKernelGGL(k_uqg_count, dim3(kMaxTiles, y), dim3(kEmitThreads), 0, st, J);
  hipLaunchKernelGGL(k_uqg_scan, dim3(1, y), dim3(kMaxTiles), 0, st, J);
  hipLaunchKernelGGL(k_uqg_emit, dim3(kMaxTiles, y), dim3(kEmitThreads), 0, st, J);
  hipLaunchKernelGGL(k_uqg_far, dim3(1, y), dim3(kFarThreads), 0, st, J);
  if (n_max > 0) {
    const unsigned g = static_cast<unsigned>(std::min<int64_t>(kGrid, (n_max + 255) / 256));
    hipLaunchKernelGGL(k_uqg_tail, dim3(g, y), dim3(256), 0, st, J);
  }
  return check_launch(fn);
}

}  // namespace
}  // namespace hgd

using namespace hgd;

extern "C" size_t hgd_unique_workspace_size(int64_t n) {
  const size_t s = n > 0 ? sort_path_bytes(n) : 0;
  const size_t d = dev_path_bytes(n > 0 ? n : 1);
  return std::max(s, d);
}

extern "C" hgd_status hgd_unique_i64(const int64_t* keys, int64_t n, int64_t* out,
                                     int64_t* n_out, void* ws, size_t wsb, void* stream) {
  clear_error();
  HGD_REQUIRE(n == 0 || keys, "hgd_unique_i64: null keys");
  return unique_bitmap(I64Src{keys}, n, out, n_out, ws, wsb, as_stream(stream), "hgd_unique_i64");
}

extern "C" hgd_status hgd_unique_trunc_f32(const float* x, int64_t n, int64_t* out,
                                           int64_t* n_out, void* ws, size_t wsb, void* stream) {
  clear_error();
  HGD_REQUIRE(n == 0 || x, "hgd_unique_trunc_f32: null x");
  return unique_bitmap(TruncSrc{x}, n, out, n_out, ws, wsb, as_stream(stream),
                       "hgd_unique_trunc_f32");
}

extern "C" hgd_status hgd_unique_sort_i64(const int64_t* keys, int64_t n, int64_t* out,
                                          int64_t* n_out, void* ws, size_t wsb, void* stream) {
  clear_error();
  HGD_REQUIRE(n == 0 || keys, "hgd_unique_sort_i64: null keys");
  return unique_sort(I64Src{keys}, keys, n, out, n_out, ws, wsb, as_stream(stream),
                     "hgd_unique_sort_i64");
}

extern "C" hgd_status hgd_unique_sort_trunc_f32(const float* x, int64_t n, int64_t* out,
                                                int64_t* n_out, void* ws, size_t wsb,
                                                void* stream) {
  clear_error();
  HGD_REQUIRE(n == 0 || x, "hgd_unique_sort_trunc_f32: null x");
  return unique_sort(TruncSrc{x}, nullptr, n, out, n_out, ws, wsb, as_stream(stream),
                     "hgd_unique_sort_trunc_f32");
}

extern "C" hgd_status hgd_unique_dev_i64(const int64_t* keys, int64_t n, int64_t* out,
                                         int64_t* n_out, void* ws, size_t wsb, void* stream) {
  clear_error();
  HGD_REQUIRE(n == 0 || keys, "hgd_unique_dev_i64: null keys");
  return unique_bitmap<I64Src, true>(I64Src{keys}, n, out, n_out, ws, wsb, as_stream(stream),
                                     "hgd_unique_dev_i64");
}

extern "C" hgd_status hgd_unique_dev_trunc_f32(const float* x, int64_t n, int64_t* out,
                                               int64_t* n_out, void* ws, size_t wsb,
                                               void* stream) {
  clear_error();
  HGD_REQUIRE(n == 0 || x, "hgd_unique_dev_trunc_f32: null x");
  return unique_bitmap<TruncSrc, true>(TruncSrc{x}, n, out, n_out, ws, wsb, as_stream(stream),
                                       "hgd_unique_dev_trunc_f32");
}

extern "C" hgd_status hgd_unique_dev_group(const hgd_unique_job* jobs, int32_t count,
                                           void* stream) {
  clear_error();
  return unique_group(jobs, count, as_stream(stream), "hgd_unique_dev_group");
}
