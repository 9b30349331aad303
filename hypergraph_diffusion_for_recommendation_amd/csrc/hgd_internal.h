// Internal helpers shared by the libhgd translation units (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "../../include/hgd.h"

namespace hgd {

// Thread-local last-error text returned by hgd_get_last_error_string().
extern thread_local char g_last_error[512];

inline hgd_status fail(hgd_status st, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
  return st;
}

inline void clear_error() { g_last_error[0] = '\0'; }

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Checks the most recent launch; turns a HIP error into HGD_ERR_HIP with context.
inline hgd_status check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(HGD_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
  return HGD_OK;
}

#define HGD_REQUIRE(cond, ...)                                   \
  do {                                                           \
    if (!(cond)) return ::hgd::fail(HGD_ERR_INVALID_ARG, __VA_ARGS__); \
  } while (0)

#define HGD_HIP(call)                                                              \
  do {                                                                             \
    hipError_t _e = (call);                                                        \
    if (_e != hipSuccess)                                                          \
      return ::hgd::fail(HGD_ERR_HIP, "%s failed: %s", #call, hipGetErrorString(_e)); \
  } while (0)

constexpr int kBlock = 256;

inline unsigned grid_for(int64_t n, int per_block = kBlock) {
  int64_t g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return static_cast<unsigned>(g);
}

inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

// out[c] = Σ_{s < S} P[s·W + c] for c < W, summed in a fixed order (deterministic): 16 waves per
// block each sum a contiguous slice of s for 64 columns, then the slices are added in order
// (reduce.hip). Used for split-K and per-block partials.
hgd_status sum_rows(const float* P, int64_t S, int64_t W, float* out, hipStream_t st);

// Several independent column sums (up to 4) in one launch, each exactly as sum_rows.
struct SumRowsJob {
  const float* P;
  int64_t S, W;
  float* out;
  float scale;  // 0 = off: out = sum × scale
};
hgd_status sum_rows_jobs(const SumRowsJob* jobs, int n, hipStream_t st);

// HGD_TUNE_ROWGEMM_BLOCKS (linear.hip): 0 restores the default.
void set_row_gemm_max_blocks(int blocks);
// HGD_TUNE_SPLITK_ROWS (linear.hip): rows per split-K slice, 0 restores the sizing rule.
void set_splitk_rows(int rows);
// HGD_TUNE_GEMM_EXACT (linear.hip): 1 = the exact f32-MFMA products only (no split-bf16).
void set_gemm_exact(int exact);
// HGD_TUNE_X3_COLS (linear.hip): column-slice width of the split-bf16 row GEMM (0, 64 or 128).
void set_x3_cols(int cols);
// HGD_TUNE_X3_SPLITK (linear.hip): 0 = the f32-MFMA split-K weight gradient even when split-bf16
// products are on, 1 = split-bf16, 2 = by shape (default).
void set_x3_splitk(int mode);
// HGD_TUNE_X3S_TILES (linear.hip): 16-column tiles per wave of the staged row GEMM (0 = default).
void set_x3s_tiles(int tiles);
// HGD_TUNE_X3P_QUEUE (linear.hip): 1 = k_splitk_x3p's queue form (per-buffer counters).
void set_x3p_queue(int queue);
// HGD_TUNE_P2P_SEGMENT_MB / HGD_TUNE_P2P_CACHED (p2p.hip): layout of later hgd_p2p_create calls.
void set_p2p_segment_mb(int mb);
void set_p2p_cached(int cached);
void set_p2p_grid(int grid);
// HGD_TUNE_CPU_RNG_THREADS (torch_rng.cpp): threads of the split keep-mask draw (0 = auto).
void set_cpu_rng_threads(int threads);
bool cpu_rng_jump_selfcheck(int64_t refills);

}  // namespace hgd
