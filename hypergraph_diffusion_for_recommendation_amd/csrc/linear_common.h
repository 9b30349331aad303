// Shared by the dense-product translation units (linear.hip, linear_x3s.hip): the row-GEMM
// descriptors, the split-bf16 helpers and the staged kernel's per-K launchers (not part of the ABI).
#pragma once

#include "device_util.h"
#include "hgd_internal.h"

namespace hgd {
namespace lin {

__device__ __forceinline__ f32x4 relu_mask(f32x4 v, f32x4 m) {
  return f32x4{m.x > 0.f ? v.x : 0.f, m.y > 0.f ? v.y : 0.f, m.z > 0.f ? v.z : 0.f,
               m.w > 0.f ? v.w : 0.f};
}

// 16 wait states after an MFMA chain whose results are read next, placed where the chain ends.
// hipcc (ROCm 7.2) inserts the MFMA→VALU read hazard's wait states only when the first read is
// in the same basic block as the MFMA; across a branch (a runtime epilogue flag) the staged row
// GEMM read its accumulators too early at NTW = 1 (tests/diag: N = 16 products off by O(1)).
// Two s_nop 7 cover the 16-pass chains here; they cost 16 cycles per tile.
__device__ __forceinline__ void mfma_drain() { asm volatile("s_nop 7\n\ts_nop 7" ::: "memory"); }

__device__ __forceinline__ bool al16_dev(const float* p, int64_t ld) {
  return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && ld % 4 == 0;
}

struct RowGemm {
  const float* A;     // [rows, K]
  int64_t lda;
  const float* mask;  // optional [rows, K]: A ⊙ (mask > 0)
  int64_t ldm;
  const float* B;     // Bm[k][n] = B[k * bsk + n * bsn]
  int64_t bsk, bsn;
  const float* bias;  // [N] or NULL
  int32_t relu;
  float* Y;
  int64_t ldy;
  int64_t rows;
  int32_t K, N;
  int32_t accumulate;  // Y += product (the bias / ReLU apply to the product alone)
  // forward epilogue after the bias / ReLU: nn.Dropout on the product (keep-bit of element
  // row·N + col from dropout_keep4(*drop_seed, ·), kept values × drop_scale), and a
  // second store Y2 = Y + res (the residual add after an ED-HNN block)
  const uint64_t* drop_seed;
  float drop_keep;
  float drop_scale;
  const float* res;
  int64_t ldres;
  float* Y2;
  int64_t ldy2;
  // A as its nonzero pattern (a > 0 ? 1 : 0: the binary incidence of a dense learned hypergraph,
  // nonzero(H > 0) of EquivSetGNN2.py:105-133); row_inv: the product's rows scaled by
  // 1 / max(Σ_k A[r, k], 1) (the scatter mean over a vertex's hyperedges) and that factor stored
  int32_t binarize_a;
  float* row_inv;
  const float* b_row_count;  // Bm row k × 1 / max(b_row_count[k], 1) (hyperedge means)
  float b_scale;             // 0 = off: Bm × b_scale (fl(W · s), as a pre-scaled W)
  // nn.Dropout on A as it is loaded (element row·K + k of the a_drop_seed draw, kept × scale):
  // the ED-HNN block's input dropout inside lin_in (EquivSetGNN2.py:91-92)
  const uint64_t* a_drop_seed;
  float a_drop_keep;
  float a_drop_scale;
};

// Up to two independent products of the same K, N and mask mode in ONE launch (HCCF's user and
// item halves of the learned-hypergraph products): blocks [0, nb0) take p[0], the rest p[1],
// each with its own grid-stride loop. The launch count, not the bytes, bounds these 10 MB
// products (profiles/r02_small_kernels).
struct RowGemmGroup {
  RowGemm p[2];
  int32_t count;
  int32_t nb0;
  int32_t nbt;  // row-block workgroups of the group (nb0 + the second's); a multiple of 8 when
                // ny > 1
  int32_t ny;   // 64-column slices of N
};

// Workgroup → (row block, column slice). With one slice it is blockIdx.x. With ny > 1 the slices
// of a row block get flat ids f, f + 8, …: the dispatcher places consecutive ids on consecutive
// XCDs, so ids 8 apart share one XCD's L2 and start together — the slices walk the same row tiles
// in the same order, so the other slices' A tile (and ReLU mask) reads hit that L2. At
// 144,242 × 128 → 128: forward 53.4 → 52.3 µs, backward-data 78.1 → 75.3 µs against the
// slice-major order (profiles/r02_linear/xcd_pairing_ab.txt); the second read was mostly served
// by the Infinity Cache already — these products are bound by the MFMA issue, not by A.
__device__ __forceinline__ void row_block_of(const RowGemmGroup& g, int& bxg, int& y) {
  const int f = static_cast<int>(blockIdx.x);
  if (g.ny == 1) {
    bxg = f;
    y = 0;
    return;
  }
  const int grp = f / (8 * g.ny), r = f % (8 * g.ny);
  y = r / 8;
  bxg = grp * 8 + r % 8;
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x4 mfma_bf16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// x = hi + mid + lo exactly: hi = bf16_rn(x), mid = bf16_rn(x - hi), lo = bf16_rn(x - hi - mid)
__device__ __forceinline__ void split3(const float (&v)[8], bf16x8& hi, bf16x8& mid, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 a = static_cast<__bf16>(v[j]);
    const float r1 = v[j] - static_cast<float>(a);
    const __bf16 b = static_cast<__bf16>(r1);
    const float r2 = r1 - static_cast<float>(b);
    hi[j] = a;
    mid[j] = b;
    lo[j] = static_cast<__bf16>(r2);
  }
}

// The same for four values (a float4 piece of a row): three bf16x4 terms.
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void split3x4(f32x4 x, bf16x4& hi, bf16x4& mid, bf16x4& lo) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const __bf16 a = static_cast<__bf16>(x[j]);
    const float r1 = x[j] - static_cast<float>(a);
    const __bf16 b = static_cast<__bf16>(r1);
    hi[j] = a;
    mid[j] = b;
    lo[j] = static_cast<__bf16>(r1 - static_cast<float>(b));
  }
}

// acc += W·x over one k step: small terms first (they are added to the running sum while it is
// small); with hi-only x (binarized 0/1 rows) the mid / lo products are zero and skipped
__device__ __forceinline__ f32x4 mfma_x3(const bf16x8& w0, const bf16x8& w1, const bf16x8& w2,
                                         const bf16x8& x0, const bf16x8& x1, const bf16x8& x2,
                                         f32x4 acc, bool x_hi_only) {
  acc = mfma_bf16(w2, x0, acc);
  if (!x_hi_only) {
    acc = mfma_bf16(w1, x1, acc);
    acc = mfma_bf16(w0, x2, acc);
  }
  acc = mfma_bf16(w1, x0, acc);
  if (!x_hi_only) acc = mfma_bf16(w0, x1, acc);
  return mfma_bf16(w0, x0, acc);
}

// Buffer-resource access (raw buffer, byte range [0, bytes) from base): an offset at or past the
// range reads zeros without touching memory and drops a store. The staged kernel addresses a row
// block through one resource per stage (base = the block's first row) with per-lane offsets that
// do not change from stage to stage: no 64-bit address arithmetic or row clamps per access, and
// no store under a branch (hipcc's vmcnt accounting then stays exact across the ring).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kBufOff = 0x80000000u;  // an offset outside every range used here
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, static_cast<int>(bytes),
                                           0x00020000);
}
__device__ __forceinline__ f32x4 buf_ld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ void buf_st4(__amdgpu_buffer_rsrc_t r, uint32_t off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, 0);
}

// row GEMM epilogue kinds of the staged split-bf16 kernel (linear_x3s.hip)
constexpr int kEpiPlain = 0, kEpiRes = 1, kEpiAcc = 2;

// The staged split-bf16 row GEMM for K = 32·KQ (linear_x3s.hip, one translation unit per KQ so
// that the instantiations compile in parallel).
// tiles: 16-column tiles per wave (HGD_TUNE_X3S_TILES; 0 = default)
template <int KQ>
hgd_status launch_x3s_k(const RowGemmGroup& g, int tiles, hipStream_t st, const char* fn);

}  // namespace lin
}  // namespace hgd
