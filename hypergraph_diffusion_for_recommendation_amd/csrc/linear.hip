// The skinny Linear layers around the ED-HNN hops ("lin_in GEMM + ReLU …
// Linear (MFMA at d ≥ 64)"): nn.Linear(d, d) over N ≫ d rows — lin_in (EquivSetGNN2.py:93-94,
// EquivSetGNN.py:88-89) and the MLP layers (model/layers/MLP.py:109-117). The library GEMMs the
// reference gets for these shapes are tiled for square problems: the profile of the Yelp-shaped
// block (profiles/r01_edhnn_yelp) shows the weight gradient [64 × 64] = dYᵀ·X with K = 69,716
// rows taking 0.20 ms (4 workgroups on a 256-CU chip) and the forward 30 µs for 36 MB.
//
// All three products run on the f32-input MFMA v_mfma_f32_16x16x4_f32 (exact f32 products and
// sums, at the f32 vector rate) with operands loaded straight from HBM as float4 rows:
//
//  * row GEMM (forward Y = relu?(X·Wᵀ + b), backward-data dX = (dY ⊙ [Y > 0])·W): W's 64-column
//    slice is staged once per workgroup through LDS into registers (K/16 × 16 floats per lane),
//    then each wave streams 16-row tiles (grid-stride, next tile's loads in flight during the
//    current tile's MFMAs), so every input row is read once and every output row written once
//    (≈ 16 flop per byte at d = 64, where the f32 MFMA and HBM rates meet). Lane l loads float4
//    X[r0 + (l&15)][4(l>>4) + 16q]; MFMA step (q, c) then multiplies k = 4(l>>4) + 16q + c — a
//    fixed permutation of k that the W fragments follow, so the rows need no LDS or shuffles.
//  * split-K weight GEMM (dW = (dY ⊙ mask)ᵀ·X, db = Σ dY ⊙ mask): the rows are cut into S slices
//    (one workgroup each, ≤ 1024); lane l loads float4 row fragments of both operands and the 16
//    MFMAs of a 4-row step produce the whole 64 × 64 tile with (m, n) = (4i + t, 4j + u)
//    permuted; the 4 waves are combined in LDS in wave order, the S slice partials by sum_rows in
//    slice order. No atomics: results are bitwise reproducible.
#include <algorithm>
#include <type_traits>

#include "linear_common.h"

namespace hgd {
namespace {

using namespace lin;


constexpr int kRowGemmMaxBlocks = 512;  // default of HGD_TUNE_ROWGEMM_BLOCKS
int g_row_gemm_max_blocks = kRowGemmMaxBlocks;
constexpr int kSplitKResident = 512;
int g_splitk_rows = 0;  // HGD_TUNE_SPLITK_ROWS (0: sized by splits_for / tn_splits)




// K = 16·KQ; NT = live 16-column tiles of a 64-column slice (N < 64: no MFMAs on zero columns);
// MASK: A ⊙ (mask > 0). BLDS: the B fragments are read from LDS (k-contiguous, one 16-byte read
// per 4 MFMAs) instead of being held in registers — at K = 128 the register copy (128 VGPRs)
// left one wave per SIMD and the 144 k × 128 × 128 forward ran at 0.32 of the f32 MFMA peak
template <int KQ, int NT, bool MASK, bool BLDS>
__device__ __forceinline__ void row_gemm_body(const RowGemmGroup& grp) {
  int bxg, ys;
  row_block_of(grp, bxg, ys);
  const bool second = grp.count > 1 && bxg >= grp.nb0;
  const RowGemm p = second ? grp.p[1] : grp.p[0];
  const int bx = bxg - (second ? grp.nb0 : 0);
  const int nbx = grp.count > 1 ? (second ? grp.nbt - grp.nb0 : grp.nb0) : grp.nbt;
  constexpr int K = 16 * KQ;
  constexpr int LDB = 65;           // padded row: the k-contiguous staging writes spread banks
  constexpr int PER = K * 64 / 256;  // staged floats per thread
  // 16-row sub-tiles per wave iteration. One: at two (32-row super-tiles) the operand ping-pong
  // held 64-128 VGPRs and the 69,716 × 64 forward ran 18.4 µs against 16.8 µs for the masked
  // backward-data form with one, which moves 1.5× the bytes (profiles/r02_small_kernels)
  constexpr int SUB = 1;
  constexpr int LDK = K + 4;         // BLDS row of 64 + K floats: 16-byte reads spread banks
  __shared__ float sB[BLDS ? 64 * LDK : K * LDB];  // Bm[k][n0 + nl] (BLDS: at nl·LDK + k)
  // per-wave 16 × 64 output tile, transposed through LDS so that full tiles leave as 16-byte
  // row stores (1 KB = four whole rows per instruction) instead of 64-byte column pieces
  constexpr int LDY = 68;
  __shared__ float sY[NT == 4 && !MASK ? 4 * 16 * LDY : 1];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int i16 = lane & 15;
  const int h = lane >> 4;
  const int n0 = ys * 64;
  const int nt = min(NT, (p.N - n0) / 16);  // live 16-column tiles of this slice (uniform)
  const int64_t tiles = (p.rows + 16 * SUB - 1) / (16 * SUB);  // super-tiles
  const int64_t stride = static_cast<int64_t>(nbx) * 4;
  int64_t tile = static_cast<int64_t>(bx) * 4 + wave;
  // Unconditional raw loads (the compiler then counts them exactly in its vmcnt waits): rows
  // past the end are clamped to the last row and their results never stored; the ReLU mask is
  // applied when the tile is consumed.
  // res rows of the tile (the Y2 = Y + res store) are fetched with its A rows: loaded in the
  // epilogue they were a dependent HBM round trip per tile (W's store of an ED-HNN block at
  // 144 k × 128: 133 µs with, 65 µs without the residual)
  float rv0[NT][4], rv1[NT][4];
  auto load = [&](int64_t tl, f32x4 (&a)[SUB][KQ], f32x4 (&m)[SUB][KQ], float (&rv)[NT][4]) {
    tl = tl < tiles ? tl : tiles - 1;
    if (!MASK && p.Y2) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int64_t row = tl * 16 + 4 * h + r;
          row = row < p.rows ? row : p.rows - 1;
          const int col = t < nt ? n0 + 16 * t + i16 : n0 + i16;
          rv[t][r] = p.res[row * p.ldres + col];
        }
    }
#pragma unroll
    for (int s = 0; s < SUB; ++s) {
      int64_t ra = tl * 16 * SUB + 16 * s + i16;
      ra = ra < p.rows ? ra : p.rows - 1;
#pragma unroll
      for (int q = 0; q < KQ; ++q) a[s][q] = ld4(p.A + ra * p.lda + 4 * h + 16 * q);
      if constexpr (MASK) {
#pragma unroll
        for (int q = 0; q < KQ; ++q) m[s][q] = ld4(p.mask + ra * p.ldm + 4 * h + 16 * q);
      }
    }
  };
  // the first tile's row loads go out before the W staging below: on small problems (one or
  // two tiles per wave) the two HBM round trips then overlap instead of adding up
  f32x4 a0[SUB][KQ], a1[SUB][KQ], m0v[SUB][KQ], m1v[SUB][KQ];
  if (tile < tiles) load(tile, a0, m0v, rv0);
  {
    // all loads first (independent, in flight together), then the LDS writes
    float tmp[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int e = threadIdx.x + 256 * j;
      const int k = p.bsk == 1 ? e % K : e / 64;
      const int nl = p.bsk == 1 ? e / K : e % 64;
      const int n = n0 + nl < p.N ? n0 + nl : p.N - 1;
      tmp[j] = p.B[static_cast<int64_t>(k) * p.bsk + static_cast<int64_t>(n) * p.bsn];
      if (n0 + nl >= p.N) tmp[j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int e = threadIdx.x + 256 * j;
      const int k = p.bsk == 1 ? e % K : e / 64;
      const int nl = p.bsk == 1 ? e / K : e % 64;
      if constexpr (BLDS) {
        // the operand scales as in the register path: × 1/max(count, 1), then × b_scale
        float v = tmp[j];
        if (p.b_row_count) v *= 1.f / fmaxf(p.b_row_count[k], 1.f);
        if (p.b_scale != 0.f) v *= p.b_scale;
        sB[nl * LDK + k] = v;
      } else {
        sB[k * LDB + nl] = tmp[j];
      }
    }
  }
  __syncthreads();
  float bf[BLDS ? 1 : KQ][4][NT];
  if constexpr (!BLDS) {
#pragma unroll
  for (int q = 0; q < KQ; ++q)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int t = 0; t < NT; ++t) bf[q][c][t] = sB[(4 * h + 16 * q + c) * LDB + 16 * t + i16];
  if (p.b_row_count) {  // fl(Bm[k][n] · fl(1 / max(count, 1))): the scaled-B product, bitwise
#pragma unroll
    for (int q = 0; q < KQ; ++q)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float inv = 1.f / fmaxf(p.b_row_count[4 * h + 16 * q + c], 1.f);
#pragma unroll
        for (int t = 0; t < NT; ++t) bf[q][c][t] *= inv;
      }
  }
  if (p.b_scale != 0.f) {
#pragma unroll
    for (int q = 0; q < KQ; ++q)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int t = 0; t < NT; ++t) bf[q][c][t] *= p.b_scale;
  }
  }
  float bias_v[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) bias_v[t] = (p.bias && t < nt) ? p.bias[n0 + 16 * t + i16] : 0.f;

  const uint64_t drop_seed = p.drop_seed ? *p.drop_seed : 0ull;
  const uint32_t drop_thr = dropout_threshold(p.drop_keep);
  const uint64_t a_seed = p.a_drop_seed ? *p.a_drop_seed : 0ull;
  const uint32_t a_thr = dropout_threshold(p.a_drop_keep);
  auto compute = [&](int64_t tile, f32x4 (&a)[SUB][KQ], const f32x4 (&m)[SUB][KQ],
                     const float (&rv)[NT][4]) {
#pragma unroll
    for (int s = 0; s < SUB; ++s) {
      if (p.a_drop_seed) {  // the float4 at k = 4h + 16q is one keep group (K % 16 == 0)
        const uint32_t e0 = static_cast<uint32_t>(tile * 16 * SUB + 16 * s + i16) *
                            static_cast<uint32_t>(p.K);
#pragma unroll
        for (int q = 0; q < KQ; ++q)
          a[s][q] = dropout_apply4(a[s][q], a_seed, (e0 + 4 * h + 16 * q) >> 2, a_thr,
                                   p.a_drop_scale);
      }
      if constexpr (MASK) {
#pragma unroll
        for (int q = 0; q < KQ; ++q) a[s][q] = relu_mask(a[s][q], m[s][q]);
      }
      if (!MASK && p.binarize_a) {
#pragma unroll
        for (int q = 0; q < KQ; ++q)
#pragma unroll
          for (int c = 0; c < 4; ++c) a[s][q][c] = a[s][q][c] > 0.f ? 1.f : 0.f;
      }
      f32x4 acc[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (BLDS) {
#pragma unroll
        for (int q = 0; q < KQ; ++q) {
          f32x4 bq[NT];
#pragma unroll
          for (int t = 0; t < NT; ++t)
            bq[t] = *reinterpret_cast<const f32x4*>(&sB[(16 * t + i16) * LDK + 4 * h + 16 * q]);
#pragma unroll
          for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t] = mfma4(a[s][q][c], bq[t][c], acc[t]);
        }
      } else {
#pragma unroll
        for (int q = 0; q < KQ; ++q)
#pragma unroll
          for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t] = mfma4(a[s][q][c], bf[q][c][t], acc[t]);
      }
      mfma_drain();
      const int64_t r0 = tile * 16 * SUB + 16 * s;
      if (!MASK && p.row_inv) {
        // Σ_k A[row i16][k]: this lane's 4·KQ columns, then the four lanes h of the row
        float rs = 0.f;
#pragma unroll
        for (int q = 0; q < KQ; ++q) rs += (a[s][q][0] + a[s][q][1]) + (a[s][q][2] + a[s][q][3]);
        rs += __shfl_xor(rs, 16);
        rs += __shfl_xor(rs, 32);
        const float inv = 1.f / fmaxf(rs, 1.f);
        if (h == 0 && n0 == 0 && r0 + i16 < p.rows) p.row_inv[r0 + i16] = inv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float sc = __shfl(inv, 4 * h + r);  // lane 4h + r holds output row 4h + r's
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[t][r] *= sc;
        }
      }
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[t][r] + bias_v[t];
          acc[t][r] = (p.relu && v < 0.f) ? 0.f : v;
        }
      if (p.drop_seed) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const uint32_t e = static_cast<uint32_t>(r0 + 4 * h + r) * static_cast<uint32_t>(p.N) +
                               static_cast<uint32_t>(n0 + 16 * t + i16);
            acc[t][r] = dropout_keep(drop_seed, e, drop_thr) ? acc[t][r] * p.drop_scale : 0.f;
          }
      }
      // (the masked backward-data form keeps the direct stores: 7 % slower at d = 64 through LDS)
      if constexpr (NT == 4 && !MASK) {
        if (nt == NT && r0 + 16 <= p.rows && !p.accumulate && al16_dev(p.Y, p.ldy) &&
            (!p.Y2 || al16_dev(p.Y2, p.ldy2))) {
          float* w = sY + wave * 16 * LDY;
          auto wave_store = [&](float* dst, int64_t ld, bool add_res) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                w[(4 * h + r) * LDY + 16 * t + i16] = add_res ? acc[t][r] + rv[t][r] : acc[t][r];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int rr = 4 * j + h;
              const f32x4 v = *reinterpret_cast<const f32x4*>(&w[rr * LDY + 4 * i16]);
              *reinterpret_cast<f32x4*>(dst + (r0 + rr) * ld + n0 + 4 * i16) = v;
            }
          };
          wave_store(p.Y, p.ldy, false);
          if (p.Y2) wave_store(p.Y2, p.ldy2, true);
          continue;
        }
      }
      float* yb = p.Y + n0 + i16;
      if (p.accumulate) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (t < nt && r0 + 4 * h + r < p.rows)
              acc[t][r] += yb[(r0 + 4 * h + r) * p.ldy + 16 * t];
      }
      if (nt == NT && r0 + 16 <= p.rows) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) yb[(r0 + 4 * h + r) * p.ldy + 16 * t] = acc[t][r];
      } else {
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (t < nt && r0 + 4 * h + r < p.rows)
              yb[(r0 + 4 * h + r) * p.ldy + 16 * t] = acc[t][r];
      }
      if (!MASK && p.Y2) {
        float* y2 = p.Y2 + n0 + i16;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (t < nt && r0 + 4 * h + r < p.rows)
              y2[(r0 + 4 * h + r) * p.ldy2 + 16 * t] = acc[t][r] + rv[t][r];
      }
    }
  };
  if (tile >= tiles) return;  // after the block's barrier: every wave took part in it
  // ping-pong buffers: the next super-tile's loads are in flight during this one's MFMAs
  while (tile < tiles) {
    load(tile + stride, a1, m1v, rv1);
    __builtin_amdgcn_sched_barrier(0);
    compute(tile, a0, m0v, rv0);
    __builtin_amdgcn_sched_barrier(0);
    tile += stride;
    if (tile >= tiles) break;
    load(tile + stride, a0, m0v, rv0);
    __builtin_amdgcn_sched_barrier(0);
    compute(tile, a1, m1v, rv1);
    __builtin_amdgcn_sched_barrier(0);
    tile += stride;
  }
}

// Unmasked (forward) products: the compiler's own register budget (2-3 waves per SIMD).
template <int KQ, int NT, bool BLDS>
__global__ __launch_bounds__(256) void k_row_gemm(RowGemmGroup grp) {
  row_gemm_body<KQ, NT, false, BLDS>(grp);
}

// Masked (backward-data) products: held to two waves per SIMD. At K = 128 the operand and mask
// ping-pong took 259 registers (one wave per SIMD) and dX = (dY ⊙ [Y > 0])·W at 144,242 × 128
// ran 75 µs; at two waves it runs 61 µs (profiles/r02_linear/occupancy_masked.txt).
template <int KQ, int NT, bool BLDS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_row_gemm_masked(
    RowGemmGroup grp) {
  row_gemm_body<KQ, NT, true, BLDS>(grp);
}

// ---------------------------------------------------------------------------------------------
// Split-bf16 row GEMM (the default for K a multiple of 32). The f32-input MFMA runs at 1/16 of
// the bf16 rate, so at d = 128 the exact-f32 row GEMM is bound by the MFMA (4.73 GFLOP at
// 157 TF = 30 µs for 144 k rows) and not by its 148 MB of HBM traffic (18.5 µs). Here every f32
// operand is cut EXACTLY into three bf16 terms, x = x0 + x1 + x2 (round-to-nearest, each
// residual exact in f32: 8 + 8 + 8 significant bits cover the 24 of an f32), and
// a·b = Σ_{i+j ≤ 2} a_i·b_j takes six v_mfma_f32_16x16x32_bf16 (bf16 products are exact in f32,
// accumulated in f32; the dropped a1·b2 + a2·b1 + a2·b2 are < 2^-23·|a·b|): 2.7× the f32 MFMA
// rate, error ≈ that of the f32 fmaf chain (1e-7 of Σ|a·b|; not bitwise the same sums, so
// hgd_set_tuning(HGD_TUNE_GEMM_EXACT, 1) keeps the f32-MFMA kernel for bitwise fmaf chains).
// Non-finite operands (and |x| within 2^-9 of FLT_MAX, whose bf16 rounding overflows) give NaN.
//
// Layout: W's slice (K × up to 128 columns) is split once per workgroup into three bf16 planes
// in LDS, each 16-byte fragment where the lane that feeds it to the MFMA reads it
// (ds_read_b128, conflict-free). The MFMA takes W as its A operand and the activation rows as
// its B operand, so the 16 × 16 result tile holds one ROW per lane (column l & 15 of D) and four
// consecutive output columns per lane (rows 4(l >> 4) + r of D): every lane stores float4 pieces
// of its own row — the epilogue (bias, ReLU, dropout, residual, row_inv) needs no transpose.
// A wave owns 16-row tiles over ALL ≤ 128 columns, so every activation row is read once.
// Lane (i, g) loads row i's floats [32q + 4g, +4) and [32q + 16 + 4g, +4) for k step q: MFMA k
// index 8g + j is that permutation of the true k, which the W fragments follow.

int g_gemm_exact = 0;  // HGD_TUNE_GEMM_EXACT


// Column slices of 16·NT columns: 128 (NT = 8, 512-thread workgroups: two waves per SIMD with
// W's 96 KB of planes filling the LDS) or 64 (NT = 4, 256 threads, 48 KB of planes: several
// workgroups per CU; the second slice's A reads hit the XCD's L2, row_block_of). HGD_TUNE_X3_COLS.
int g_x3_cols = 0;  // 0: default
int g_x3s_tiles = 0;  // HGD_TUNE_X3S_TILES (0: default)
int g_x3_splitk = 2;  // HGD_TUNE_X3_SPLITK: 1 split-bf16 weight gradient, 0 f32 MFMA, 2 auto
int g_x3p_queue = 0;  // HGD_TUNE_X3P_QUEUE: 1 = the queue form of k_splitk_x3p

// The split-bf16 split-K kernel pays for its six products with one k step in flight per slice:
// at 144,242 × 128 it ran 79 µs against the f32-MFMA kernel's 59 µs; at 69,716 × 64 19.9 against
// 21.1, at 31,668 × 64 16.0 against 13.1 (profiles/r03_linear). Auto: split-bf16 for outputs of
// at most 64 × 64 over at least 49,152 rows. The same rule sizes the workspace and launches.
bool use_x3_splitk(const hgd_gemm_tn_desc* d, int count) {
  if (g_gemm_exact || g_x3_splitk == 0) return false;
  if (g_x3_splitk == 1) return true;
  int64_t rows = 0;
  for (int i = 0; i < count; ++i) {
    if (d[i].rows <= 0) continue;
    if (d[i].M > 64 || d[i].N > 64) return false;
    rows += d[i].rows;
  }
  return rows >= 49152;
}

// NT: 16-column tiles of a ≤ 128-column slice (1, 2, 4 or 8). Tiles past the live nt (N not a
// multiple of 16·NT) are staged as zeros and computed like the others — only their stores are
// skipped — so the MFMA stream has no branches; binarized rows likewise run all six products.
template <int KQ, int NT, bool MASK, int THREADS>
__global__ __launch_bounds__(THREADS) void k_row_gemm_x3(RowGemmGroup grp) {
  extern __shared__ __attribute__((aligned(16))) char x3_smem[];
  bf16x8* sW = reinterpret_cast<bf16x8*>(x3_smem);  // [3][NT][KQ][64]
  float* sBias = reinterpret_cast<float*>(sW + 3 * NT * KQ * 64);  // [NT·16]
  int bxg, ys;
  row_block_of(grp, bxg, ys);
  const bool second = grp.count > 1 && bxg >= grp.nb0;
  const RowGemm p = second ? grp.p[1] : grp.p[0];  // a copy: its fields live in registers
  const int bx = bxg - (second ? grp.nb0 : 0);
  const int nbx = grp.count > 1 ? (second ? grp.nbt - grp.nb0 : grp.nb0) : grp.nbt;
  constexpr int WAVES = THREADS / 64;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int i16 = lane & 15;
  const int g = lane >> 4;
  const int n0 = ys * 16 * NT;
  const int nt = min(NT, (p.N - n0) / 16);
  const int64_t tiles = (p.rows + 15) / 16;
  const int64_t stride = static_cast<int64_t>(nbx) * WAVES;
  int64_t tile = static_cast<int64_t>(bx) * WAVES + wave;

  // activation rows of a tile (+ its mask rows)
  auto load = [&](int64_t tl, f32x4 (&a)[KQ][2], f32x4 (&m)[KQ][2]) {
    tl = tl < tiles ? tl : tiles - 1;
    int64_t row = tl * 16 + i16;
    row = row < p.rows ? row : p.rows - 1;
    const float* ar = p.A + row * p.lda + 4 * g;
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      a[q][0] = ld4(ar + 32 * q);
      a[q][1] = ld4(ar + 32 * q + 16);
    }
    if constexpr (MASK) {
      const float* mr = p.mask + row * p.ldm + 4 * g;
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        m[q][0] = ld4(mr + 32 * q);
        m[q][1] = ld4(mr + 32 * q + 16);
      }
    }
  };
  f32x4 a0[KQ][2], a1[KQ][2], m0v[KQ][2], m1v[KQ][2];
  if (tile < tiles) load(tile, a0, m0v);

  // W's slice → three bf16 planes in fragment order (+ the bias slice): every fragment's eight
  // loads first (in flight together), then the splits and the LDS stores
  {
    constexpr int FRAGS = NT * KQ * 64;
    constexpr int FR = (FRAGS + THREADS - 1) / THREADS;
    float v[FR][8];
#pragma unroll
    for (int r = 0; r < FR; ++r) {
      const int f = threadIdx.x + THREADS * r;
      const int L = f & 63, q = (f >> 6) % KQ, t = (f >> 6) / KQ;
      const int gg = L >> 4;
      const bool live = f < FRAGS && t < nt;
      const int n = live ? n0 + 16 * t + (L & 15) : 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 32 * (live ? q : 0) + (j < 4 ? 4 * gg + j : 16 + 4 * gg + (j - 4));
        v[r][j] = p.B[static_cast<int64_t>(k) * p.bsk + static_cast<int64_t>(n) * p.bsn];
        if (p.b_row_count) v[r][j] *= 1.f / fmaxf(p.b_row_count[k], 1.f);
        if (p.b_scale != 0.f) v[r][j] *= p.b_scale;
        if (!live) v[r][j] = 0.f;
      }
    }
#pragma unroll
    for (int r = 0; r < FR; ++r) {
      const int f = threadIdx.x + THREADS * r;
      if (f < FRAGS) {
        const int L = f & 63, q = (f >> 6) % KQ, t = (f >> 6) / KQ;
        bf16x8 h, md, lo;
        split3(v[r], h, md, lo);
        sW[((0 * NT + t) * KQ + q) * 64 + L] = h;
        sW[((1 * NT + t) * KQ + q) * 64 + L] = md;
        sW[((2 * NT + t) * KQ + q) * 64 + L] = lo;
      }
    }
  }
  for (int c = threadIdx.x; c < NT * 16; c += THREADS)
    sBias[c] = (p.bias && c < nt * 16) ? p.bias[n0 + c] : 0.f;
  __syncthreads();
  if (tile >= tiles) return;  // after the block's barrier

  const uint64_t drop_seed = p.drop_seed ? *p.drop_seed : 0ull;
  const uint32_t drop_thr = dropout_threshold(p.drop_keep);
  const uint64_t a_seed = p.a_drop_seed ? *p.a_drop_seed : 0ull;
  const uint32_t a_thr = dropout_threshold(p.a_drop_keep);
  auto compute = [&](int64_t tl, const f32x4 (&a)[KQ][2], const f32x4 (&m)[KQ][2]) {
    const int64_t row = tl * 16 + i16;
    const bool live = row < p.rows;
    // the residual pieces of the Y2 store, requested before this tile's MFMAs (≈ 1 µs of them)
    f32x4 rv[NT];
    if (!MASK && p.Y2) {
      const float* rr = p.res + (live ? row : p.rows - 1) * p.ldres + n0 + 4 * g;
#pragma unroll
      for (int t = 0; t < NT; ++t) rv[t] = ld4(rr + 16 * (t < nt ? t : 0));
    }
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float rs = 0.f;
    // W fragments double-buffered: group (q, t + 1)'s three LDS reads are issued before group
    // (q, t)'s six MFMAs, so the reads' latency hides behind them
    bf16x8 wf[2][3];
    auto read_w = [&](int q, int t, bf16x8 (&w)[3]) {
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) w[pl] = sW[((pl * NT + t) * KQ + q) * 64 + lane];
    };
    read_w(0, 0, wf[0]);
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      f32x4 x0 = a[q][0], x1 = a[q][1];
      if (p.a_drop_seed) {  // each float4 piece is one keep group of the input dropout
        const uint32_t e0 = static_cast<uint32_t>(row) * static_cast<uint32_t>(p.K) + 32 * q + 4 * g;
        x0 = dropout_apply4(x0, a_seed, e0 >> 2, a_thr, p.a_drop_scale);
        x1 = dropout_apply4(x1, a_seed, (e0 + 16) >> 2, a_thr, p.a_drop_scale);
      }
      if constexpr (MASK) {
        x0 = relu_mask(x0, m[q][0]);
        x1 = relu_mask(x1, m[q][1]);
      } else {
        if (p.binarize_a) {
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            x0[c] = x0[c] > 0.f ? 1.f : 0.f;
            x1[c] = x1[c] > 0.f ? 1.f : 0.f;
          }
        }
        if (p.row_inv) rs += ((x0.x + x0.y) + (x0.z + x0.w)) + ((x1.x + x1.y) + (x1.z + x1.w));
      }
      const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      bf16x8 xh, xm, xl;
      split3(v, xh, xm, xl);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int cur = (q * NT + t) & 1;
        if (t + 1 < NT) read_w(q, t + 1, wf[cur ^ 1]);
        else if (q + 1 < KQ) read_w(q + 1, 0, wf[cur ^ 1]);
        acc[t] = mfma_x3(wf[cur][0], wf[cur][1], wf[cur][2], xh, xm, xl, acc[t], false);
      }
    }
    mfma_drain();
    // lane (i16, g): row r0 + i16, columns n0 + 16t + 4g + c in acc[t][c]
    if (!MASK && p.row_inv) {
      rs += __shfl_xor(rs, 16);
      rs += __shfl_xor(rs, 32);
      const float inv = 1.f / fmaxf(rs, 1.f);
      if (g == 0 && n0 == 0 && live) p.row_inv[row] = inv;
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] *= inv;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(&sBias[16 * t + 4 * g]);
      const int col = n0 + 16 * t + 4 * g;
      f32x4 v = acc[t] + b4;
      if (p.relu) {
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = v[c] < 0.f ? 0.f : v[c];
      }
      if (p.drop_seed) {  // the lane's four columns are one keep group (N % 16 == 0)
        const uint32_t e = static_cast<uint32_t>(row) * static_cast<uint32_t>(p.N) +
                           static_cast<uint32_t>(col);
        v = dropout_apply4(v, drop_seed, e >> 2, drop_thr, p.drop_scale);
      }
      if (!live || t >= nt) continue;
      float* y = p.Y + row * p.ldy + col;
      if (p.accumulate) v += ld4(y);
      *reinterpret_cast<f32x4*>(y) = v;
      if (!MASK && p.Y2) *reinterpret_cast<f32x4*>(p.Y2 + row * p.ldy2 + col) = v + rv[t];
    }
  };
  while (tile < tiles) {
    load(tile + stride, a1, m1v);
    __builtin_amdgcn_sched_barrier(0);
    compute(tile, a0, m0v);
    __builtin_amdgcn_sched_barrier(0);
    tile += stride;
    if (tile >= tiles) break;
    load(tile + stride, a0, m0v);
    __builtin_amdgcn_sched_barrier(0);
    compute(tile, a1, m1v);
    __builtin_amdgcn_sched_barrier(0);
    tile += stride;
  }
}


struct SplitK {
  const float* A;  // [rows, M] (dY)
  int64_t lda;
  const float* mask;
  int64_t ldm;
  const float* B;  // [rows, N] (X)
  int64_t ldb;
  int64_t rows;
  int32_t M, N;
  int64_t rows_per_split;
  float* part;       // [S, M·N]
  float* part_bias;  // [S, M] or NULL
  int32_t binarize_a;  // A as its nonzero pattern (a > 0 ? 1 : 0)
  const float* b_row_scale;  // [rows] or NULL: B row × scale on load
  const uint64_t* b_drop_seed;  // nn.Dropout on B as it is loaded (element row·N + n), before
  float b_drop_keep;            // b_row_scale
  float b_drop_scale;
};

struct SplitKGroup {  // as RowGemmGroup: blocks [0, nb0) along x are p[0]'s row slices
  SplitK p[2];
  int32_t count;
  int32_t nb0;
};

template <bool MASK>
__global__ __launch_bounds__(256) void k_splitk_tn(SplitKGroup grp) {
  const bool second = grp.count > 1 && static_cast<int>(blockIdx.x) >= grp.nb0;
  const SplitK p = second ? grp.p[1] : grp.p[0];
  const int64_t bx = static_cast<int64_t>(blockIdx.x) - (second ? grp.nb0 : 0);
  __shared__ float s_acc[4][64 * 64];
  __shared__ float s_bias[4][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int i16 = lane & 15;
  const int h = lane >> 4;
  const int m0 = blockIdx.y * 64;
  const int n0 = blockIdx.z * 64;
  const int64_t k_begin = bx * p.rows_per_split;
  const int64_t k_end = min(p.rows, k_begin + p.rows_per_split);
  const bool mcol = m0 + 4 * i16 < p.M;
  const bool ncol = n0 + 4 * i16 < p.N;
  const int mc = mcol ? m0 + 4 * i16 : m0;  // clamped (valid) columns; zeroed at consume
  const int nc = ncol ? n0 + 4 * i16 : n0;
  const bool want_bias = p.part_bias != nullptr && blockIdx.z == 0;
  f32x4 acc[4][4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[t][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum[4] = {0.f, 0.f, 0.f, 0.f};
  const uint64_t b_seed = p.b_drop_seed ? *p.b_drop_seed : 0ull;
  const uint32_t b_thr = dropout_threshold(p.b_drop_keep);

  // 4-row steps per wave per batch (loads of batch b+1 overlap b's MFMAs); 8 steps held 212-256
  // VGPRs (one wave per SIMD), 4 steps allow two
  constexpr int U = 4;
  // Unconditional loads from clamped rows (exact vmcnt accounting by the compiler); rows past
  // k_end and columns past M / N are zeroed when consumed.
  auto load = [&](int64_t kb, f32x4 (&a)[U], f32x4 (&b)[U], f32x4 (&m)[U]) {
#pragma unroll
    for (int s = 0; s < U; ++s) {
      int64_t kr = kb + 16 * s + h;
      kr = kr < k_end ? kr : k_begin;
      a[s] = ld4(p.A + kr * p.lda + mc);
      if constexpr (MASK) m[s] = ld4(p.mask + kr * p.ldm + mc);
      b[s] = ld4(p.B + kr * p.ldb + nc);
      if (p.b_drop_seed)  // the float4 at column nc is one keep group (N % 16 == 0)
        b[s] = dropout_apply4(b[s], b_seed,
                              static_cast<uint32_t>(kr * p.N + nc) >> 2, b_thr, p.b_drop_scale);
      if (p.b_row_scale) {  // fl(B · scale), as a pre-scaled B would hold it
        const float sc = p.b_row_scale[kr];
        b[s] = f32x4{b[s].x * sc, b[s].y * sc, b[s].z * sc, b[s].w * sc};
      }
    }
  };
  auto compute = [&](int64_t kb, const f32x4 (&ca)[U], const f32x4 (&cb)[U],
                     const f32x4 (&cm)[U]) {
#pragma unroll
    for (int s = 0; s < U; ++s) {
      const bool ok = kb + 16 * s + h < k_end;
      f32x4 av = ca[s], bv = cb[s];
      if constexpr (MASK) av = relu_mask(av, cm[s]);
      if (p.binarize_a)
        av = f32x4{av.x > 0.f ? 1.f : 0.f, av.y > 0.f ? 1.f : 0.f, av.z > 0.f ? 1.f : 0.f,
                   av.w > 0.f ? 1.f : 0.f};
      if (!(ok && mcol)) av = f32x4{0.f, 0.f, 0.f, 0.f};
      if (!(ok && ncol)) bv = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[t][u] = mfma4(av[t], bv[u], acc[t][u]);
      if (want_bias) {
#pragma unroll
        for (int t = 0; t < 4; ++t) bsum[t] += av[t];
      }
    }
  };
  // ping-pong buffers (no loop-carried copies, which the compiler would hoist into the MFMA
  // stream together with a full vmcnt wait)
  f32x4 a0[U], b0[U], m0v[U], a1[U], b1[U], m1v[U];
  int64_t kb = k_begin + 4 * wave;
  load(kb, a0, b0, m0v);
  while (kb < k_end) {
    load(kb + 16 * U, a1, b1, m1v);
    __builtin_amdgcn_sched_barrier(0);
    compute(kb, a0, b0, m0v);
    __builtin_amdgcn_sched_barrier(0);
    kb += 16 * U;
    if (kb >= k_end) break;
    load(kb + 16 * U, a0, b0, m0v);
    __builtin_amdgcn_sched_barrier(0);
    compute(kb, a1, b1, m1v);
    __builtin_amdgcn_sched_barrier(0);
    kb += 16 * U;
  }
  mfma_drain();
  // acc[t][u] lane (i16, h) reg r: m_local = 4·(4h + r) + t, n_local = 4·i16 + u
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        s_acc[wave][(4 * (4 * h + r) + t) * 64 + 4 * i16 + u] = acc[t][u][r];
  if (want_bias) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      bsum[t] += __shfl_xor(bsum[t], 16);
      bsum[t] += __shfl_xor(bsum[t], 32);
      if (h == 0) s_bias[wave][4 * i16 + t] = bsum[t];
    }
  }
  __syncthreads();
  const int64_t MN = static_cast<int64_t>(p.M) * p.N;
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int ml = e >> 6, nl = e & 63;
    if (m0 + ml < p.M && n0 + nl < p.N) {
      const float v = ((s_acc[0][e] + s_acc[1][e]) + s_acc[2][e]) + s_acc[3][e];
      p.part[bx * MN + static_cast<int64_t>(m0 + ml) * p.N + n0 + nl] = v;
    }
  }
  if (want_bias && threadIdx.x < 64 && m0 + static_cast<int>(threadIdx.x) < p.M) {
    const int ml = threadIdx.x;
    p.part_bias[bx * p.M + m0 + ml] =
        ((s_bias[0][ml] + s_bias[1][ml]) + s_bias[2][ml]) + s_bias[3][ml];
  }
}

// Split-bf16 form of k_splitk_tn (see k_row_gemm_x3 for the numerics). The reduction runs over
// rows, so an MFMA's k index is a row: lane (i16, g) loads rows 8g + j (j < 8) of a 32-row step
// as float4 pieces of A at columns 4·i16 and float2 pieces of B at columns 2·i16; component t of
// its eight A pieces is the A fragment of MFMA (t, u) (output m = 4·i + t), component u of the B
// pieces its B fragment (n = 2·i16 + u): 4 × 2 products × 6 split terms give a 64 × 32 tile per
// 32 rows. A workgroup of 8 waves covers up to eight such tiles of the output at once (all of a
// 128 × 128 weight gradient), so every row of A and B is read from HBM once per slice — the
// 64 × 64-tile grid re-read each operand once per tile of the other (296 MB for a 148 MB
// product at d = 128); with fewer tiles than waves the rows are dealt to P = 8 / tiles phases,
// combined in LDS in phase order. Every operand of a step is split before the next step's loads
// are issued, so those loads fly during this step's MFMAs.
constexpr int kX3SplitKThreads = 512;
constexpr int kX3SplitKResident = 256;  // workgroups of one resident round (one per CU)

__host__ __device__ constexpr int x3_tiles_per_wg(int tiles) {
  return tiles % 8 == 0 ? 8 : (tiles % 4 == 0 ? 4 : (tiles % 2 == 0 ? 2 : 1));
}

template <bool MASK>
__global__ __launch_bounds__(kX3SplitKThreads) void k_splitk_tn_x3(SplitKGroup grp) {
  const bool second = grp.count > 1 && static_cast<int>(blockIdx.x) >= grp.nb0;
  const SplitK p = second ? grp.p[1] : grp.p[0];
  const int64_t bx = static_cast<int64_t>(blockIdx.x) - (second ? grp.nb0 : 0);
  constexpr int WAVES = kX3SplitKThreads / 64;
  __shared__ float s_acc[WAVES][64 * 32];
  __shared__ float s_bias[WAVES][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int i16 = lane & 15;
  const int g = lane >> 4;
  const int tiles_h = (p.N + 31) / 32;
  const int Qg = x3_tiles_per_wg(((p.M + 63) / 64) * tiles_h);
  const int P = WAVES / Qg;
  const int slot = wave % Qg, phase = wave / Qg;
  const int tile = static_cast<int>(blockIdx.y) * Qg + slot;
  const int m0 = (tile / tiles_h) * 64;
  const int n0 = (tile % tiles_h) * 32;
  const int64_t k_begin = bx * p.rows_per_split;
  const int64_t k_end = min(p.rows, k_begin + p.rows_per_split);
  const bool mcol = m0 + 4 * i16 < p.M;
  const bool ncol = n0 + 2 * i16 < p.N;
  const int mc = mcol ? m0 + 4 * i16 : m0;
  const int nc = ncol ? n0 + 2 * i16 : n0;
  const bool want_bias = p.part_bias != nullptr && n0 == 0;
  const bool hi_only = p.binarize_a != 0;
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  f32x4 acc[4][2];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u) acc[t][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum[4] = {0.f, 0.f, 0.f, 0.f};
  const uint64_t b_seed = p.b_drop_seed ? *p.b_drop_seed : 0ull;
  const uint32_t b_thr = dropout_threshold(p.b_drop_keep);

  f32x4 a[8], m[8];
  f32x2 b[8];
  float sc[8];
  auto load = [&](int64_t kb) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int64_t kr = kb + 8 * g + j;
      kr = kr < k_end ? kr : k_begin;
      a[j] = ld4(p.A + kr * p.lda + mc);
      if constexpr (MASK) m[j] = ld4(p.mask + kr * p.ldm + mc);
      b[j] = *reinterpret_cast<const f32x2*>(p.B + kr * p.ldb + nc);
      if (p.b_row_scale) sc[j] = p.b_row_scale[kr];
    }
  };
  const int64_t step = 32 * P;
  int64_t kb = k_begin + 32 * phase;
  if (kb < k_end) load(kb);
  while (kb < k_end) {
    bool ok[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) ok[j] = kb + 8 * g + j < k_end;
    bf16x8 bs[2][3], as[4][3];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float x = b[j][u];
        if (p.b_drop_seed) {  // elements nc, nc + 1 are half of one keep group
          const uint32_t e = static_cast<uint32_t>((kb + 8 * g + j) * p.N + nc + u);
          x = dropout_keep(b_seed, e, b_thr) ? x * p.b_drop_scale : 0.f;
        }
        if (p.b_row_scale) x *= sc[j];  // fl(B · scale), as a pre-scaled B would hold it
        v[j] = (ok[j] && ncol) ? x : 0.f;
      }
      split3(v, bs[u][0], bs[u][1], bs[u][2]);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float x = a[j][t];
        if constexpr (MASK) x = m[j][t] > 0.f ? x : 0.f;
        if (hi_only) x = x > 0.f ? 1.f : 0.f;
        v[j] = (ok[j] && mcol) ? x : 0.f;
      }
      if (want_bias) bsum[t] += ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
      split3(v, as[t][0], as[t][1], as[t][2]);
    }
    kb += step;
    if (kb < k_end) load(kb);  // in flight during this step's MFMAs
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        // D = A·B (rows m, columns n); binarized A: its mid / lo products are zero, skipped
        f32x4 c = acc[t][u];
        if (!hi_only) {
          c = mfma_bf16(as[t][2], bs[u][0], c);
          c = mfma_bf16(as[t][1], bs[u][1], c);
        }
        c = mfma_bf16(as[t][0], bs[u][2], c);
        if (!hi_only) c = mfma_bf16(as[t][1], bs[u][0], c);
        c = mfma_bf16(as[t][0], bs[u][1], c);
        acc[t][u] = mfma_bf16(as[t][0], bs[u][0], c);
      }
    __builtin_amdgcn_sched_barrier(0);
  }
  mfma_drain();
  // acc[t][u] lane (i16, g) reg r: m_local = 4·(4g + r) + t, n_local = 2·i16 + u
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        s_acc[wave][(4 * (4 * g + r) + t) * 32 + 2 * i16 + u] = acc[t][u][r];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    bsum[t] += __shfl_xor(bsum[t], 16);
    bsum[t] += __shfl_xor(bsum[t], 32);
    if (g == 0) s_bias[wave][4 * i16 + t] = bsum[t];
  }
  __syncthreads();
  const int64_t MN = static_cast<int64_t>(p.M) * p.N;
  for (int e = threadIdx.x; e < Qg * 64 * 32; e += kX3SplitKThreads) {
    const int q = e / (64 * 32), el = e % (64 * 32);
    const int tq = static_cast<int>(blockIdx.y) * Qg + q;
    const int mq = (tq / tiles_h) * 64 + el / 32, nq = (tq % tiles_h) * 32 + el % 32;
    if (mq < p.M && nq < p.N) {
      float v = s_acc[q][el];
      for (int ph = 1; ph < P; ++ph) v += s_acc[ph * Qg + q][el];
      p.part[bx * MN + static_cast<int64_t>(mq) * p.N + nq] = v;
    }
  }
  if (p.part_bias != nullptr) {
    for (int e = threadIdx.x; e < Qg * 64; e += kX3SplitKThreads) {
      const int q = e / 64, ml = e % 64;
      const int tq = static_cast<int>(blockIdx.y) * Qg + q;
      const int mq = (tq / tiles_h) * 64 + ml;
      if (tq % tiles_h == 0 && mq < p.M) {
        float v = s_bias[q][ml];
        for (int ph = 1; ph < P; ++ph) v += s_bias[ph * Qg + q][ml];
        p.part_bias[bx * p.M + mq] = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Weight gradient with producer waves (dW = (dY ⊙ mask)ᵀ·X, db = Σ dY ⊙ mask; M = N = 128): the
// row-GEMM's structure applied to split-K. A workgroup owns one row slice and the whole 128 × 128
// output, so each operand row is read ONCE (the 64 × 64-tile f32 kernel read both twice: 2.0× the
// algorithmic bytes, profiles/r03_linear/pmc). At 128 × 128, 16 waves (at 64 × 64, 12):
//
//  * 8 (4) producer waves stream 32-row stages of both operands (the first half dY and its ReLU
//    mask, the second X) through a register ring two stages deep: each thread loads a 4-row × 4-column
//    block (float4 per row; a wave instruction covers two full 512-B rows), applies the mask /
//    binarization (dY) or the input dropout and row scale (X), splits every column's four values
//    into the three bf16 terms and writes them as 8-byte halves of the MFMA fragments, both
//    operands TRANSPOSED in LDS (fragment (column c, k-group g) = rows 8g .. 8g + 7 of column c);
//  * 8 consumer waves multiply the previous stage: wave (mp, nq) owns output tiles
//    TM·mp .. + TM - 1 × TN·nq .. + TN - 1 (16 × 16 each; TM × TN = 2 × 4 at 128, 1 × 2 at 64)
//    and runs 6 split-bf16 MFMAs per tile per stage;
//  * fragment unit (c, g) sits at 16-B unit c·4 + (g ^ ((c >> 1) & 3)) and producer b writes
//    its columns in the order (c + (cb >> 1)) & 3: conflict-free ds_read_b128 (lane groups
//    {0–3,12–15,20–27}, …) and ds_write_b64 (16 consecutive lanes) on gfx950 (searched
//    exhaustively over the candidate swizzles);
//  * the slice's partial tile and column sums go to `part` / `part_bias` as the other split-K
//    kernels' (summed by sum_rows in slice order).
// MT = 16-column output tiles per side (8: 128 × 128, 16 waves; 4: 64 × 64, 8 consumer + 4
// producer waves, each consumer two tiles).
constexpr int kX3pResident = 256;  // one workgroup per CU
template <int MT>
struct X3P {
  static constexpr int C4 = 4 * MT;                     // 4-column blocks of an operand row
  static constexpr int PROD = 2 * 8 * C4;               // producer threads (both operands)
  static constexpr int THREADS = 512 + PROD;            // + 8 consumer waves
  static constexpr int TM = MT / 4, TN = MT / 2;        // output tiles of a consumer wave
  static constexpr size_t PLANE = static_cast<size_t>(MT) * 16 * 4 * 16;  // one operand, one term
  static constexpr size_t LDS = 2 * 2 * 3 * PLANE;      // [buffer][operand][term]
  // the queue form: three buffers and, after them, the stage counters full[3] / empty[3]
  static constexpr size_t LDS_Q = 3 * 2 * 3 * PLANE + 64;
  static constexpr uint32_t PROD_WAVES = PROD / 64;
};

__device__ __forceinline__ int x3p_unit(int c, int g) { return c * 4 + (g ^ ((c >> 1) & 3)); }

// QUEUE: the producer and consumer sides meet through per-buffer counters instead of one
// workgroup barrier per stage (three LDS buffers; a producer wave waits only until the consumers
// have READ the stage three back, a consumer wave only until the 8 producer waves have written its
// stage — the sides drift by up to two stages). The barrier form couples all 16 waves every 32
// rows: PMC put them 49 % parked at that barrier (profiles/r03_linear/pmc).
template <int MT, bool MASK, bool QUEUE>
__global__ __launch_bounds__(X3P<MT>::THREADS) void k_splitk_x3p(SplitKGroup grp) {
  using C = X3P<MT>;
  constexpr size_t kX3pPlane = C::PLANE;
  extern __shared__ __attribute__((aligned(16))) char x3p_smem[];
  const bool second = grp.count > 1 && static_cast<int>(blockIdx.x) >= grp.nb0;
  const SplitK p = second ? grp.p[1] : grp.p[0];
  const int64_t bx = static_cast<int64_t>(blockIdx.x) - (second ? grp.nb0 : 0);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int i16 = lane & 15;
  const int g = lane >> 4;
  const int64_t k_begin = bx * p.rows_per_split;
  const int64_t k_end = min(p.rows, k_begin + p.rows_per_split);
  const int64_t n_st = k_end > k_begin ? (k_end - k_begin + 31) / 32 : 0;
  auto plane = [&](int buf, int op, int term) -> char* {
    return x3p_smem + static_cast<size_t>((buf * 2 + op) * 3 + term) * kX3pPlane;
  };
  float bsum[4] = {0.f, 0.f, 0.f, 0.f};  // dY producers: column sums of their block
  const int pt = tid - 512;              // producer thread index
  // queue form: full[b] counts producer-wave arrivals at buffer b, empty[b] consumer-wave
  // departures (monotone over the slice: stage i uses buffer i % 3 for the (i / 3)-th time)
  uint32_t* const full = reinterpret_cast<uint32_t*>(x3p_smem + 3 * 2 * 3 * kX3pPlane);
  uint32_t* const empty = full + 3;
  uint32_t* const stall = full + 6;  // set by any wave whose wait ran out (LDS_Q's spare words)
  if constexpr (QUEUE) {
    if (tid < 7) full[tid] = 0u;
    __syncthreads();
  }
  // bounded: every wave leaves the loop (the counts are reached within microseconds). A wave
  // descheduled past the bound (≈ 0.1 s: preemption, a shared GPU) would read a buffer not yet
  // filled or overwrite one in use, so a wait that runs out marks the workgroup, and its whole
  // output is written as NaN below — a loud failure, never silently wrong gradients.
  auto spin_until = [&](const uint32_t* c, uint32_t target) {
    for (uint32_t n = 0; n < (1u << 22); ++n) {
      if (__hip_atomic_load(c, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) return;
      __builtin_amdgcn_s_sleep(1);
    }
    __hip_atomic_store(stall, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  auto arrive = [&](uint32_t* c) {  // after this wave's LDS accesses of the stage
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  const int pb = pt % (8 * C::C4), gq = pb / (2 * C::C4), hh = pb & 1, cb = (pb >> 1) % C::C4;

  // one producer role (OP 0: dY [+ mask], 1: X): a loop of exactly n_st barriers
  auto produce = [&](auto op_tag) {
    constexpr int OP = decltype(op_tag)::value;
    const float* base = OP == 0 ? p.A : p.B;
    const int64_t ld = OP == 0 ? p.lda : p.ldb;
    uint32_t off[4], moff[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t r = 8 * gq + 4 * hh + j;
      off[j] = (r * static_cast<uint32_t>(ld) + 4 * cb) * 4;
      moff[j] = (r * static_cast<uint32_t>(p.ldm) + 4 * cb) * 4;
    }
    const uint64_t seed = p.b_drop_seed ? *p.b_drop_seed : 0ull;
    const uint32_t thr = dropout_threshold(p.b_drop_keep);
    constexpr int D = 2;
    f32x4 raw[D][4], rawm[D][4];
    auto load = [&](int64_t s, f32x4 (&a)[4], f32x4 (&m)[4]) {
      const int64_t r0 = k_begin + 32 * s;
      const uint32_t nr = s < n_st ? static_cast<uint32_t>(min<int64_t>(32, k_end - r0)) : 0u;
      const int64_t rb0 = nr ? r0 : 0;
      const auto rs = buf_rsrc(base + rb0 * ld, nr * static_cast<uint32_t>(ld) * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = buf_ld4(rs, off[j]);
      if constexpr (OP == 0 && MASK) {
        const auto rm = buf_rsrc(p.mask + rb0 * p.ldm, nr * static_cast<uint32_t>(p.ldm) * 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) m[j] = buf_ld4(rm, moff[j]);
      }
    };
    auto split = [&](int64_t s, int buf, const f32x4 (&a)[4], const f32x4 (&m)[4]) {
      const int64_t r0 = k_begin + 32 * s + 8 * gq + 4 * hh;  // this block's first row
      f32x4 v[4];                                              // v[j] = row j, columns 0..3
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4 x = a[j];
        if constexpr (OP == 0) {
          if constexpr (MASK) x = relu_mask(x, m[j]);
          if (p.binarize_a) {
#pragma unroll
            for (int c = 0; c < 4; ++c) x[c] = x[c] > 0.f ? 1.f : 0.f;
          }
#pragma unroll
          for (int c = 0; c < 4; ++c) bsum[c] += x[c];
        } else {
          if (p.b_drop_seed) {  // keep group of elements row·N + 4cb .. + 3
            const uint32_t e = static_cast<uint32_t>((r0 + j) * p.N + 4 * cb);
            x = dropout_apply4(x, seed, e >> 2, thr, p.b_drop_scale);
          }
        }
        v[j] = x;
      }
      if constexpr (OP == 1) {
        if (p.b_row_scale) {  // fl(B · scale), as a pre-scaled B would hold it
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int64_t r = r0 + j < k_end ? r0 + j : k_begin;
            v[j] *= p.b_row_scale[r];
          }
        }
      }
#pragma unroll
      for (int c0 = 0; c0 < 4; ++c0) {
        const int c = (c0 + (cb >> 1)) & 3;
        const f32x4 col{v[0][c], v[1][c], v[2][c], v[3][c]};
        bf16x4 t0, t1, t2;
        split3x4(col, t0, t1, t2);
        const size_t o = static_cast<size_t>(x3p_unit(4 * cb + c, gq)) * 16 + 8 * hh;
        *reinterpret_cast<bf16x4*>(plane(buf, OP, 0) + o) = t0;
        *reinterpret_cast<bf16x4*>(plane(buf, OP, 1) + o) = t1;
        *reinterpret_cast<bf16x4*>(plane(buf, OP, 2) + o) = t2;
      }
    };
#pragma unroll
    for (int d = 0; d < D; ++d) load(d, raw[d], rawm[d]);
    if constexpr (QUEUE) {
      // stage i: wait until buffer i % 3 is free (its previous stage read), split, arrive, then
      // refill the ring slot with stage i + D
      auto qstep = [&](int64_t i, f32x4 (&a)[4], f32x4 (&m)[4]) {
        const int b = static_cast<int>(i % 3);
        if (i >= 3) spin_until(empty + b, 8u * static_cast<uint32_t>(i / 3));
        split(i, b, a, m);
        arrive(full + b);
        load(i + D, a, m);
      };
      int64_t i0 = 0;
      for (; i0 + D <= n_st; i0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) qstep(i0 + d, raw[d], rawm[d]);
      }
#pragma unroll
      for (int d = 0; d < D; ++d)
        if (i0 + d < n_st) qstep(i0 + d, raw[d], rawm[d]);
      return;
    }
    if (n_st > 0) {
      split(0, 0, raw[0], rawm[0]);
      load(D, raw[0], rawm[0]);
    }
    auto pstep = [&](int64_t i, bool has_next, f32x4 (&a)[4], f32x4 (&m)[4]) {
      __syncthreads();
      if (has_next) {
        split(i + 1, static_cast<int>((i + 1) & 1), a, m);
        load(i + 1 + D, a, m);
      }
    };
    int64_t i0 = 0;
    for (; i0 + D < n_st; i0 += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) pstep(i0 + d, true, raw[(d + 1) % D], rawm[(d + 1) % D]);
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
      if (i0 + d < n_st) pstep(i0 + d, i0 + d + 1 < n_st, raw[(d + 1) % D], rawm[(d + 1) % D]);
    }
  };

  f32x4 acc[C::TM][C::TN];
#pragma unroll
  for (int t = 0; t < C::TM; ++t)
#pragma unroll
    for (int u = 0; u < C::TN; ++u) acc[t][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int mp = wave & 3, nq = (wave >> 2) & 1;
  if (tid >= 512 + 8 * C::C4) {
    produce(std::integral_constant<int, 1>{});
  } else if (wave >= 8) {
    produce(std::integral_constant<int, 0>{});
  } else if constexpr (QUEUE) {
    for (int64_t i = 0; i < n_st; ++i) {
      const int b = static_cast<int>(i % 3);
      spin_until(full + b, C::PROD_WAVES * static_cast<uint32_t>(i / 3 + 1));
      bf16x8 af[C::TM][3], bfr[C::TN][3];
#pragma unroll
      for (int t = 0; t < C::TM; ++t)
#pragma unroll
        for (int tm = 0; tm < 3; ++tm)
          af[t][tm] = *reinterpret_cast<const bf16x8*>(
              plane(b, 0, tm) +
              static_cast<size_t>(x3p_unit(16 * (C::TM * mp + t) + i16, g)) * 16);
#pragma unroll
      for (int u = 0; u < C::TN; ++u)
#pragma unroll
        for (int tm = 0; tm < 3; ++tm)
          bfr[u][tm] = *reinterpret_cast<const bf16x8*>(
              plane(b, 1, tm) +
              static_cast<size_t>(x3p_unit(16 * (C::TN * nq + u) + i16, g)) * 16);
      arrive(empty + b);  // the fragments are in registers: the buffer may be refilled
#pragma unroll
      for (int u = 0; u < C::TN; ++u)
#pragma unroll
        for (int t = 0; t < C::TM; ++t)
          acc[t][u] = mfma_x3(af[t][0], af[t][1], af[t][2], bfr[u][0], bfr[u][1], bfr[u][2],
                              acc[t][u], false);
    }
  } else {
    for (int64_t i = 0; i < n_st; ++i) {
      __syncthreads();
      const int buf = static_cast<int>(i & 1);
      bf16x8 af[C::TM][3];
#pragma unroll
      for (int t = 0; t < C::TM; ++t)
#pragma unroll
        for (int tm = 0; tm < 3; ++tm)
          af[t][tm] = *reinterpret_cast<const bf16x8*>(
              plane(buf, 0, tm) +
              static_cast<size_t>(x3p_unit(16 * (C::TM * mp + t) + i16, g)) * 16);
#pragma unroll
      for (int u = 0; u < C::TN; ++u) {
        bf16x8 bf[3];
#pragma unroll
        for (int tm = 0; tm < 3; ++tm)
          bf[tm] = *reinterpret_cast<const bf16x8*>(
              plane(buf, 1, tm) +
              static_cast<size_t>(x3p_unit(16 * (C::TN * nq + u) + i16, g)) * 16);
#pragma unroll
        for (int t = 0; t < C::TM; ++t)
          acc[t][u] = mfma_x3(af[t][0], af[t][1], af[t][2], bf[0], bf[1], bf[2], acc[t][u], false);
      }
    }
  }
  mfma_drain();
  __syncthreads();  // the planes are free: column sums of the dY producers through LDS
  constexpr int M = 16 * MT;
  float* s_b = reinterpret_cast<float*>(x3p_smem);  // [4 k-groups · 2 halves][M]
  if (tid >= 512 && tid < 512 + 8 * C::C4) {
#pragma unroll
    for (int c = 0; c < 4; ++c) s_b[(2 * gq + hh) * M + 4 * cb + c] = bsum[c];
  }
  const int64_t MN = static_cast<int64_t>(p.M) * p.N;
  bool poisoned = false;
  if constexpr (QUEUE)
    poisoned = __hip_atomic_load(stall, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0u;
  const float nan = __builtin_nanf("");
  if (wave < 8) {
    // acc[t][u] lane (i16, g) register r: m = 16(TM·mp + t) + 4g + r, n = 16(TN·nq + u) + i16
#pragma unroll
    for (int t = 0; t < C::TM; ++t)
#pragma unroll
      for (int u = 0; u < C::TN; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 16 * (C::TM * mp + t) + 4 * g + r, n = 16 * (C::TN * nq + u) + i16;
          p.part[bx * MN + static_cast<int64_t>(m) * p.N + n] = poisoned ? nan : acc[t][u][r];
        }
  }
  __syncthreads();
  if (p.part_bias != nullptr && tid < M) {
    float v = 0.f;
    for (int q = 0; q < 8; ++q) v += s_b[q * M + tid];
    p.part_bias[bx * p.M + tid] = poisoned ? nan : v;
  }
}

bool al16(const void* p, int64_t ld) {
  return p == nullptr || (reinterpret_cast<uintptr_t>(p) % 16 == 0 && ld % 4 == 0);
}

// Blocks per product: one per 4 16-row tiles up to the 512 workgroups resident at once; a group
// of two shares that budget in proportion to the rows.
void blocks_for(const int64_t* rows, int count, int64_t* bx) {
  int64_t tiles[2] = {0, 0}, want[2] = {0, 0}, total = 0;
  for (int i = 0; i < count; ++i) {
    tiles[i] = (rows[i] + 15) / 16;
    want[i] = (tiles[i] + 3) / 4;
    total += want[i];
  }
  for (int i = 0; i < count; ++i) {
    bx[i] = want[i];
    if (total > g_row_gemm_max_blocks)
      bx[i] = std::max<int64_t>(1, want[i] * g_row_gemm_max_blocks / total);
  }
}

constexpr size_t x3_lds_bytes(int KQ, int NT) {
  return static_cast<size_t>(3 * NT * KQ * 64) * 16 + static_cast<size_t>(NT) * 16 * 4;
}

// One split-bf16 launch: as many workgroups as the tiles want, at most one resident round (the
// occupancy of this instantiation at its LDS size × the CUs), shared by a group's products in
// proportion to their rows; column slices XCD-paired as in row_block_of.
template <int KQ, int NT, bool MASK>
hgd_status launch_x3(RowGemmGroup g, hipStream_t st, const char* fn) {
  constexpr int kX3Threads = NT == 8 ? 512 : 256;
  const void* kern = reinterpret_cast<const void*>(&k_row_gemm_x3<KQ, NT, MASK, kX3Threads>);
  constexpr size_t lds = x3_lds_bytes(KQ, NT);
  static int resident = 0;
  if (resident == 0) {
    if (lds > 65536)
      HGD_HIP(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  static_cast<int>(lds)));
    int nb = 0, dev = 0, cus = 0;
    HGD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, kX3Threads, lds));
    HGD_HIP(hipGetDevice(&dev));
    HGD_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    resident = std::max(1, nb) * std::max(1, cus);
  }
  constexpr int64_t kRowsPerBlock = 16 * (kX3Threads / 64);
  int64_t want[2] = {0, 0}, total = 0;
  for (int i = 0; i < g.count; ++i) {
    want[i] = (g.p[i].rows + kRowsPerBlock - 1) / kRowsPerBlock;
    total += want[i];
  }
  g.ny = (g.p[0].N + 16 * NT - 1) / (16 * NT);
  const int64_t cap = std::max<int64_t>(1, resident / g.ny);
  int64_t bx[2] = {0, 0};
  for (int i = 0; i < g.count; ++i) {
    bx[i] = total > cap ? std::max<int64_t>(1, want[i] * cap / total) : want[i];
    if (g.ny > 1) bx[i] = (bx[i] + 7) / 8 * 8;
  }
  g.nb0 = static_cast<int32_t>(bx[0]);
  g.nbt = static_cast<int32_t>(bx[0] + bx[1]);
  const dim3 grid(static_cast<unsigned>(g.nbt) * static_cast<unsigned>(g.ny));
  hipLaunchKernelGGL((k_row_gemm_x3<KQ, NT, MASK, kX3Threads>), grid, dim3(kX3Threads), lds, st,
                     g);
  return check_launch(fn);
}


template <int KQ, int NT>
hgd_status launch_x3_mask(const RowGemmGroup& g, hipStream_t st, const char* fn) {
  return g.p[0].mask ? launch_x3<KQ, NT, true>(g, st, fn) : launch_x3<KQ, NT, false>(g, st, fn);
}

template <int KQ>
hgd_status launch_x3_nt(const RowGemmGroup& g, hipStream_t st, const char* fn) {
  const int N = g.p[0].N;
  if (N <= 16) return launch_x3_mask<KQ, 1>(g, st, fn);
  if (N <= 32) return launch_x3_mask<KQ, 2>(g, st, fn);
  if (N <= 64 || g_x3_cols == 64) return launch_x3_mask<KQ, 4>(g, st, fn);  // 0 never reaches here
  return launch_x3_mask<KQ, 8>(g, st, fn);
}

// The split-bf16 kernel takes K a multiple of 32 and 16-byte aligned output rows (it stores
// float4 pieces of a row); everything else, and HGD_TUNE_GEMM_EXACT, runs the f32-MFMA kernel.
bool x3_eligible(const RowGemmGroup& g) {
  if (g_gemm_exact || g.p[0].K % 32 != 0) return false;
  for (int i = 0; i < g.count; ++i) {
    const RowGemm& p = g.p[i];
    if (!al16(p.Y, p.ldy) || !al16(p.Y2, p.ldy2) || !al16(p.res, p.ldres)) return false;
    // the staged kernel addresses a ≤ 64-row block through 32-bit byte offsets
    constexpr int64_t kLdMax = int64_t{1} << 22;
    if (p.lda >= kLdMax || p.ldm >= kLdMax || p.ldy >= kLdMax || p.ldy2 >= kLdMax ||
        p.ldres >= kLdMax)
      return false;
  }
  return true;
}

hgd_status row_gemm_group(RowGemmGroup g, hipStream_t st, const char* fn) {
  const RowGemm& p = g.p[0];
  if (g.count == 2) {
    const RowGemm& q = g.p[1];
    HGD_REQUIRE(q.K == p.K && q.N == p.N && (q.mask != nullptr) == (p.mask != nullptr),
                "%s: grouped products need equal K, N and mask mode", fn);
    if (q.rows == 0) g.count = 1;
    if (p.rows == 0) {
      g.p[0] = g.p[1];
      g.count = g.p[0].rows > 0 ? 1 : 0;
    }
  }
  if (g.count == 0 || g.p[0].rows == 0) return HGD_OK;
  if (x3_eligible(g) && g_x3_cols == 0) {
    switch (g.p[0].K / 32) {
      case 1: return launch_x3s_k<1>(g, g_x3s_tiles, st, fn);
      case 2: return launch_x3s_k<2>(g, g_x3s_tiles, st, fn);
      case 3: return launch_x3s_k<3>(g, g_x3s_tiles, st, fn);
      case 4: return launch_x3s_k<4>(g, g_x3s_tiles, st, fn);
      default: break;
    }
  }
  if (x3_eligible(g)) {
    switch (g.p[0].K / 32) {
      case 1: return launch_x3_nt<1>(g, st, fn);
      case 2: return launch_x3_nt<2>(g, st, fn);
      case 3: return launch_x3_nt<3>(g, st, fn);
      case 4: return launch_x3_nt<4>(g, st, fn);
      default: break;
    }
  }
  const int64_t rows[2] = {g.p[0].rows, g.count > 1 ? g.p[1].rows : 0};
  int64_t bx[2] = {0, 0};
  blocks_for(rows, g.count, bx);
  g.ny = (p.N + 63) / 64;
  if (g.ny > 1)  // whole groups of 8 row blocks per product (row_block_of's XCD pairing)
    for (int i = 0; i < g.count; ++i) bx[i] = (bx[i] + 7) / 8 * 8;
  g.nb0 = static_cast<int32_t>(bx[0]);
  g.nbt = static_cast<int32_t>(bx[0] + bx[1]);
  const dim3 grid(static_cast<unsigned>(g.nbt) * static_cast<unsigned>(g.ny));
  // 16-column tiles per slice: 4 for N >= 64, else N / 16 (the slice is the whole N)
  const int ntiles = g.p[0].N >= 64 ? 4 : g.p[0].N / 16;
  switch ((g.p[0].K / 16) * 8 + ntiles) {
#define HGD_CASE_NT(Q, T)                                                              \
    case Q * 8 + T:                                                                    \
      if (g.p[0].mask)                                                                 \
        hipLaunchKernelGGL((k_row_gemm_masked<Q, T, (Q > 1)>), grid, dim3(256), 0, st, g); \
      else                                                                             \
        hipLaunchKernelGGL((k_row_gemm<Q, T, (Q > 1)>), grid, dim3(256), 0, st, g);     \
      break;
#define HGD_CASE(Q) HGD_CASE_NT(Q, 1) HGD_CASE_NT(Q, 2) HGD_CASE_NT(Q, 3) HGD_CASE_NT(Q, 4)
    HGD_CASE(1) HGD_CASE(2) HGD_CASE(3) HGD_CASE(4) HGD_CASE(5) HGD_CASE(6) HGD_CASE(7)
    HGD_CASE(8)
#undef HGD_CASE
#undef HGD_CASE_NT
    default:
      return fail(HGD_ERR_UNSUPPORTED, "%s: K = %d (needs 16..128, multiple of 16)", fn,
                  g.p[0].K);
  }
  return check_launch(fn);
}

hgd_status row_gemm(const RowGemm& p, hipStream_t st, const char* fn) {
  RowGemmGroup g{};
  g.p[0] = p;
  g.count = 1;
  return row_gemm_group(g, st, fn);
}

int64_t splits_for(int64_t rows, int64_t out_tiles) {
  // ≥ 128 rows per workgroup (two 64-row batches of 4 waves × 16 rows): ≈ 250 workgroups at 32 K
  // rows (the Yelp-shaped learned-hypergraph products), where 512-row splits left 3/4 of the CUs
  // idle; at most 512 workgroups (two per CU at the kernel's two waves per SIMD), so a mid-sized
  // problem runs in one round instead of a full second round for a few leftover workgroups
  int64_t s = (rows + 127) / 128;
  // the budget counts workgroups, not slices: each slice is out_tiles workgroups (64 × 64 output
  // tiles), and the partials written and re-read are S · M · N floats — at M = N = 128, 512
  // slices were 2,048 workgroups and 34 MB of partials each way
  const int64_t cap = std::max<int64_t>(1, kSplitKResident / std::max<int64_t>(1, out_tiles));
  if (s > cap) s = cap;
  return s < 1 ? 1 : s;
}

template <int MT, bool MASK, bool QUEUE>
hgd_status launch_x3p_form(const SplitKGroup& g, int64_t Stot, hipStream_t st) {
  using C = X3P<MT>;
  constexpr size_t lds = QUEUE ? C::LDS_Q : C::LDS;
  static bool lds_set = false;
  const void* kern = reinterpret_cast<const void*>(&k_splitk_x3p<MT, MASK, QUEUE>);
  if (!lds_set) {
    if (lds > 65536)
      HGD_HIP(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  static_cast<int>(lds)));
    lds_set = true;
  }
  hipLaunchKernelGGL((k_splitk_x3p<MT, MASK, QUEUE>), dim3(static_cast<unsigned>(Stot)),
                     dim3(C::THREADS), lds, st, g);
  return HGD_OK;
}

template <int MT>
hgd_status launch_x3p(const SplitKGroup& g, int64_t Stot, hipStream_t st) {
  const bool mask = g.p[0].mask != nullptr;
  if (g_x3p_queue)
    return mask ? launch_x3p_form<MT, true, true>(g, Stot, st)
                : launch_x3p_form<MT, false, true>(g, Stot, st);
  return mask ? launch_x3p_form<MT, true, false>(g, Stot, st)
              : launch_x3p_form<MT, false, false>(g, Stot, st);
}

// The producer-wave weight gradient (k_splitk_x3p): 128 × 128 or 64 × 64 outputs whose operand rows are
// 16-byte aligned and addressable in 32-bit block offsets, by default (HGD_TUNE_X3_SPLITK = 2)
bool use_x3p_splitk(const hgd_gemm_tn_desc* d, int count) {
  if (g_gemm_exact || g_x3_splitk != 2) return false;
  int64_t rows = 0;
  constexpr int64_t kLdMax = int64_t{1} << 22;
  for (int i = 0; i < count; ++i) {
    if (d[i].rows <= 0) continue;
    if (d[i].M != d[i].N || (d[i].M != 128 && d[i].M != 64) || d[i].M != d[0].M) return false;
    if (!al16(d[i].A, d[i].lda) || !al16(d[i].B, d[i].ldb) || !al16(d[i].relu_mask, d[i].ldm))
      return false;
    if (d[i].lda >= kLdMax || d[i].ldb >= kLdMax || d[i].ldm >= kLdMax) return false;
    rows += d[i].rows;
  }
  return rows >= 4096;
}

// Row slices of each product of a split-K group (the pair shares the resident budget).
void tn_splits(const hgd_gemm_tn_desc* d, int count, int64_t* S, int64_t* per) {
  const bool x3 = use_x3_splitk(d, count);
  if (g_splitk_rows > 0) {  // HGD_TUNE_SPLITK_ROWS: fixed rows per slice
    for (int i = 0; i < count; ++i) {
      per[i] = g_splitk_rows;
      S[i] = std::max<int64_t>(1, (std::max<int64_t>(d[i].rows, 1) + per[i] - 1) / per[i]);
    }
    return;
  }
  if (use_x3p_splitk(d, count)) {  // one 1024-thread workgroup per slice, ≥ 64 rows each
    int64_t total = 0;
    for (int i = 0; i < count; ++i) {
      S[i] = std::min<int64_t>(std::max<int64_t>(1, (std::max<int64_t>(d[i].rows, 1) + 63) / 64),
                               kX3pResident);
      total += S[i];
    }
    for (int i = 0; i < count; ++i) {
      if (count > 1 && total > kX3pResident)
        S[i] = std::max<int64_t>(1, S[i] * kX3pResident / total);
      const int64_t rows = d[i].rows > 0 ? d[i].rows : 1;
      per[i] = ((rows + S[i] - 1) / S[i] + 31) / 32 * 32;  // whole 32-row stages
      S[i] = (rows + per[i] - 1) / per[i];
    }
    return;
  }
  // workgroups per slice and the resident budget: 64 × 64 tiles of 256 threads (f32 MFMA), or
  // groups of up to eight 64 × 32 tiles of 512 threads (split-bf16)
  auto wg_per_slice = [&](const hgd_gemm_tn_desc& e) -> int64_t {
    if (!x3) return static_cast<int64_t>((e.M + 63) / 64) * ((e.N + 63) / 64);
    const int t = ((e.M + 63) / 64) * ((e.N + 31) / 32);
    return t / x3_tiles_per_wg(t);
  };
  const int64_t resident = x3 ? kX3SplitKResident : kSplitKResident;
  int64_t total = 0;
  for (int i = 0; i < count; ++i) {
    if (x3) {  // ≥ 256 rows per workgroup (8 waves × 32-row steps), one resident round at most
      S[i] = std::min<int64_t>(std::max<int64_t>(1, (d[i].rows + 255) / 256),
                               std::max<int64_t>(1, resident / wg_per_slice(d[i])));
    } else {
      S[i] = splits_for(d[i].rows, wg_per_slice(d[i]));
    }
    total += S[i];
  }
  for (int i = 0; i < count; ++i) {
    const int64_t budget = std::max<int64_t>(1, resident / wg_per_slice(d[0]));
    if (count > 1 && total > budget)
      S[i] = std::max<int64_t>(1, S[i] * budget / total);
    const int64_t rows = d[i].rows > 0 ? d[i].rows : 1;
    int64_t pr = (rows + S[i] - 1) / S[i];
    per[i] = (pr + 127) / 128 * 128;  // whole 128-row steps (4 waves × 32 rows of the x3 form)
    S[i] = (rows + per[i] - 1) / per[i];
  }
}

size_t tn_part_bytes(const hgd_gemm_tn_desc& d, int64_t S) {
  return align_up(static_cast<size_t>(S) * d.M * d.N * 4);
}
size_t tn_bias_bytes(const hgd_gemm_tn_desc& d, int64_t S) {
  return d.colsum_A ? align_up(static_cast<size_t>(S) * d.M * 4) : 0;
}

hgd_status check_tn(const hgd_gemm_tn_desc& d, const char* fn) {
  HGD_REQUIRE(d.rows >= 0, "%s: negative rows", fn);
  HGD_REQUIRE(d.M % 16 == 0 && d.M >= 16 && d.N % 16 == 0 && d.N >= 16,
              "%s: M, N (%d, %d) must be positive multiples of 16", fn, d.M, d.N);
  HGD_REQUIRE(d.lda >= d.M && d.ldb >= d.N && (!d.relu_mask || d.ldm >= d.M),
              "%s: leading dimension too small", fn);
  HGD_REQUIRE(d.C, "%s: null C", fn);
  HGD_REQUIRE(!d.b_drop_seed || (d.b_drop_keep > 0.f && d.b_drop_keep <= 1.f),
              "%s: B dropout keep must be in (0, 1]", fn);
  HGD_REQUIRE(!d.b_drop_seed || d.rows * static_cast<int64_t>(d.N) <= 0xffffffffLL,
              "%s: B dropout needs rows·N < 2^32 (32-bit element counter)", fn);
  if (d.rows == 0) return HGD_OK;
  HGD_REQUIRE(d.A && d.B, "%s: null A / B", fn);
  HGD_REQUIRE(al16(d.A, d.lda) && al16(d.B, d.ldb) && al16(d.relu_mask, d.ldm),
              "%s: rows must be 16-byte aligned", fn);
  return HGD_OK;
}

hgd_status check_rows(const hgd_gemm_rows_desc& d, const char* fn) {
  HGD_REQUIRE(d.rows >= 0, "%s: negative rows", fn);
  HGD_REQUIRE(d.K % 16 == 0 && d.K >= 16 && d.K <= 128,
              "%s: K = %d must be a multiple of 16 in [16, 128]", fn, d.K);
  HGD_REQUIRE(d.N % 16 == 0 && d.N >= 16, "%s: N = %d must be a positive multiple of 16", fn,
              d.N);
  HGD_REQUIRE(d.lda >= d.K && d.ldy >= d.N && (!d.relu_mask || d.ldm >= d.K),
              "%s: leading dimension too small", fn);
  HGD_REQUIRE(!d.drop_seed || (d.drop_keep > 0.f && d.drop_keep <= 1.f),
              "%s: dropout keep must be in (0, 1]", fn);
  HGD_REQUIRE(!d.drop_seed || d.rows * static_cast<int64_t>(d.N) <= 0xffffffffLL,
              "%s: dropout needs rows·N < 2^32 (32-bit element counter)", fn);
  HGD_REQUIRE((d.res == nullptr) == (d.Y2 == nullptr), "%s: res and Y2 go together", fn);
  // the masked form is the backward-data product: its kernel carries none of the forward
  // epilogues (their registers kept it at one wave per SIMD)
  HGD_REQUIRE(!d.relu_mask || (!d.Y2 && !d.row_inv && !d.binarize_a),
              "%s: relu_mask excludes the residual, row_inv and binarize_a epilogues", fn);
  HGD_REQUIRE(!d.a_drop_seed || (d.a_drop_keep > 0.f && d.a_drop_keep <= 1.f),
              "%s: A dropout keep must be in (0, 1]", fn);
  HGD_REQUIRE(!d.a_drop_seed || d.rows * static_cast<int64_t>(d.K) <= 0xffffffffLL,
              "%s: A dropout needs rows·K < 2^32 (32-bit element counter)", fn);
  HGD_REQUIRE(!d.Y2 || (d.ldres >= d.N && d.ldy2 >= d.N), "%s: ldres / ldy2 too small", fn);
  if (d.rows == 0) return HGD_OK;
  HGD_REQUIRE(d.A && d.B && d.Y, "%s: null pointer", fn);
  HGD_REQUIRE(al16(d.A, d.lda) && al16(d.relu_mask, d.ldm), "%s: A / mask rows must be 16-byte "
              "aligned", fn);
  return HGD_OK;
}

}  // namespace

void set_row_gemm_max_blocks(int blocks) {
  g_row_gemm_max_blocks = blocks > 0 ? blocks : kRowGemmMaxBlocks;
}
void set_splitk_rows(int rows) { g_splitk_rows = rows > 0 ? rows : 0; }
void set_gemm_exact(int exact) { g_gemm_exact = exact != 0; }
void set_x3_cols(int cols) { g_x3_cols = cols; }
void set_x3_splitk(int mode) { g_x3_splitk = mode; }
void set_x3s_tiles(int tiles) { g_x3s_tiles = tiles; }
void set_x3p_queue(int queue) { g_x3p_queue = queue; }
}  // namespace hgd

extern "C" hgd_status hgd_linear_forward(const float* X, int64_t ldx, int64_t n_rows,
                                         int32_t in_features, const float* W, int64_t ldw,
                                         int32_t out_features, const float* bias, int32_t relu,
                                         float* Y, int64_t ldy, void* stream) {
  using namespace hgd;
  clear_error();
  HGD_REQUIRE(n_rows >= 0, "hgd_linear_forward: negative rows");
  HGD_REQUIRE(in_features % 16 == 0 && in_features >= 16 && in_features <= 128,
              "hgd_linear_forward: in_features %d must be a multiple of 16 in [16, 128]",
              in_features);
  HGD_REQUIRE(out_features % 16 == 0 && out_features >= 16,
              "hgd_linear_forward: out_features %d must be a positive multiple of 16",
              out_features);
  HGD_REQUIRE(ldx >= in_features && ldy >= out_features && ldw >= in_features,
              "hgd_linear_forward: leading dimension too small");
  if (n_rows == 0) return HGD_OK;
  HGD_REQUIRE(X && W && Y, "hgd_linear_forward: null pointer");
  HGD_REQUIRE(al16(X, ldx), "hgd_linear_forward: X rows must be 16-byte aligned");
  RowGemm p{};
  p.A = X;
  p.lda = ldx;
  p.B = W;  // Bm[k][n] = W[n][k]
  p.bsk = 1;
  p.bsn = ldw;
  p.bias = bias;
  p.relu = relu != 0;
  p.Y = Y;
  p.ldy = ldy;
  p.rows = n_rows;
  p.K = in_features;
  p.N = out_features;
  return row_gemm(p, as_stream(stream), "hgd_linear_forward");
}

extern "C" hgd_status hgd_linear_backward_data(const float* dY, int64_t ldy, const float* relu_out,
                                               int64_t ldr, int64_t n_rows, int32_t out_features,
                                               const float* W, int64_t ldw, int32_t in_features,
                                               float* dX, int64_t ldx, void* stream) {
  using namespace hgd;
  clear_error();
  HGD_REQUIRE(n_rows >= 0, "hgd_linear_backward_data: negative rows");
  HGD_REQUIRE(out_features % 16 == 0 && out_features >= 16 && out_features <= 128,
              "hgd_linear_backward_data: out_features %d must be a multiple of 16 in [16, 128]",
              out_features);
  HGD_REQUIRE(in_features % 16 == 0 && in_features >= 16,
              "hgd_linear_backward_data: in_features %d must be a positive multiple of 16",
              in_features);
  HGD_REQUIRE(ldy >= out_features && ldx >= in_features && ldw >= in_features &&
                  (!relu_out || ldr >= out_features),
              "hgd_linear_backward_data: leading dimension too small");
  if (n_rows == 0) return HGD_OK;
  HGD_REQUIRE(dY && W && dX, "hgd_linear_backward_data: null pointer");
  HGD_REQUIRE(al16(dY, ldy) && al16(relu_out, ldr),
              "hgd_linear_backward_data: dY / relu_out rows must be 16-byte aligned");
  RowGemm p{};
  p.A = dY;
  p.lda = ldy;
  p.mask = relu_out;
  p.ldm = ldr;
  p.B = W;  // Bm[k][n] = W[k][n]  (k = output feature, n = input feature)
  p.bsk = ldw;
  p.bsn = 1;
  p.Y = dX;
  p.ldy = ldx;
  p.rows = n_rows;
  p.K = out_features;
  p.N = in_features;
  return row_gemm(p, as_stream(stream), "hgd_linear_backward_data");
}

extern "C" size_t hgd_gemm_tn_workspace_size(const hgd_gemm_tn_desc* descs, int32_t count) {
  if (!descs || count < 1 || count > 2) return 0;
  int64_t S[2] = {0, 0}, per[2] = {0, 0};
  hgd::tn_splits(descs, count, S, per);
  size_t b = 0;
  for (int i = 0; i < count; ++i) {
    if (descs[i].rows <= 0 || descs[i].M <= 0 || descs[i].N <= 0) continue;
    b += hgd::tn_part_bytes(descs[i], S[i]) + hgd::tn_bias_bytes(descs[i], S[i]);
  }
  return b;
}

extern "C" hgd_status hgd_gemm_tn(const hgd_gemm_tn_desc* descs, int32_t count, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  using namespace hgd;
  clear_error();
  HGD_REQUIRE(descs && count >= 1 && count <= 2, "hgd_gemm_tn: 1 or 2 descriptors");
  for (int i = 0; i < count; ++i) {
    const hgd_status c = check_tn(descs[i], "hgd_gemm_tn");
    if (c != HGD_OK) return c;
  }
  if (count == 2)
    HGD_REQUIRE(descs[0].M == descs[1].M && descs[0].N == descs[1].N &&
                    (descs[0].relu_mask != nullptr) == (descs[1].relu_mask != nullptr),
                "hgd_gemm_tn: grouped products need equal M, N and mask mode");
  hipStream_t st = as_stream(stream);
  const size_t need = hgd_gemm_tn_workspace_size(descs, count);
  if (workspace_bytes < need || (need && !workspace))
    return fail(HGD_ERR_WORKSPACE, "hgd_gemm_tn: workspace %zu < required %zu", workspace_bytes,
                need);
  int64_t S[2] = {0, 0}, per[2] = {0, 0};
  tn_splits(descs, count, S, per);
  SplitKGroup g{};
  char* w = static_cast<char*>(workspace);
  int live = 0;
  for (int i = 0; i < count; ++i) {
    const hgd_gemm_tn_desc& d = descs[i];
    if (d.rows == 0) {  // an empty product: zeros
      HGD_HIP(hipMemsetAsync(d.C, 0, static_cast<size_t>(d.M) * d.N * 4, st));
      if (d.colsum_A) HGD_HIP(hipMemsetAsync(d.colsum_A, 0, static_cast<size_t>(d.M) * 4, st));
      continue;
    }
    SplitK& p = g.p[live];
    p.A = d.A;
    p.lda = d.lda;
    p.mask = d.relu_mask;
    p.ldm = d.ldm;
    p.B = d.B;
    p.ldb = d.ldb;
    p.rows = d.rows;
    p.M = d.M;
    p.N = d.N;
    p.rows_per_split = per[i];
    p.binarize_a = d.binarize_a;
    p.b_row_scale = d.b_row_scale;
    p.b_drop_seed = d.b_drop_seed;
    p.b_drop_keep = d.b_drop_keep;
    p.b_drop_scale = d.b_drop_scale;
    p.part = reinterpret_cast<float*>(w);
    w += tn_part_bytes(d, S[i]);
    p.part_bias = d.colsum_A ? reinterpret_cast<float*>(w) : nullptr;
    w += tn_bias_bytes(d, S[i]);
    if (live == 0) g.nb0 = static_cast<int32_t>(S[i]);
    ++live;
  }
  if (live == 0) return HGD_OK;
  g.count = live;
  int64_t Stot = 0;
  int li = 0;
  const hgd_gemm_tn_desc* ld[2] = {nullptr, nullptr};
  int64_t Sl[2] = {0, 0};
  for (int i = 0; i < count; ++i)
    if (descs[i].rows > 0) {
      ld[li] = &descs[i];
      Sl[li++] = S[i];
      Stot += S[i];
    }
  const dim3 grid(static_cast<unsigned>(Stot), static_cast<unsigned>((g.p[0].M + 63) / 64),
                  static_cast<unsigned>((g.p[0].N + 63) / 64));
  if (use_x3p_splitk(descs, count)) {
    hgd_status ls = g.p[0].M == 128 ? launch_x3p<8>(g, Stot, st) : launch_x3p<4>(g, Stot, st);
    if (ls != HGD_OK) return ls;
  } else if (use_x3_splitk(descs, count)) {
    const int tiles = ((g.p[0].M + 63) / 64) * ((g.p[0].N + 31) / 32);
    const dim3 gx(static_cast<unsigned>(Stot),
                  static_cast<unsigned>(tiles / x3_tiles_per_wg(tiles)));
    if (g.p[0].mask)
      hipLaunchKernelGGL((k_splitk_tn_x3<true>), gx, dim3(kX3SplitKThreads), 0, st, g);
    else
      hipLaunchKernelGGL((k_splitk_tn_x3<false>), gx, dim3(kX3SplitKThreads), 0, st, g);
  } else if (g.p[0].mask) {
    hipLaunchKernelGGL((k_splitk_tn<true>), grid, dim3(256), 0, st, g);
  } else {
    hipLaunchKernelGGL((k_splitk_tn<false>), grid, dim3(256), 0, st, g);
  }
  hgd_status s = check_launch("hgd_gemm_tn");
  if (s != HGD_OK) return s;
  // the slice partials in slice order: all sums of the group in one launch
  SumRowsJob jobs[4];
  int nj = 0;
  for (int i = 0; i < live; ++i) {
    const float sc = ld[i]->c_scale;
    jobs[nj++] = SumRowsJob{g.p[i].part, Sl[i], static_cast<int64_t>(g.p[i].M) * g.p[i].N,
                            ld[i]->C, sc};
    if (ld[i]->colsum_A)
      jobs[nj++] = SumRowsJob{g.p[i].part_bias, Sl[i], g.p[i].M, ld[i]->colsum_A, sc};
  }
  return sum_rows_jobs(jobs, nj, st);
}

extern "C" hgd_status hgd_gemm_rows(const hgd_gemm_rows_desc* descs, int32_t count, void* stream) {
  using namespace hgd;
  clear_error();
  HGD_REQUIRE(descs && count >= 1 && count <= 2, "hgd_gemm_rows: 1 or 2 descriptors");
  RowGemmGroup g{};
  for (int i = 0; i < count; ++i) {
    const hgd_gemm_rows_desc& d = descs[i];
    const hgd_status c = check_rows(d, "hgd_gemm_rows");
    if (c != HGD_OK) return c;
    RowGemm& p = g.p[i];
    p.A = d.A;
    p.lda = d.lda;
    p.mask = d.relu_mask;
    p.ldm = d.ldm;
    p.B = d.B;
    p.bsk = d.bsk;
    p.bsn = d.bsn;
    p.bias = d.bias;
    p.relu = d.relu != 0;
    p.Y = d.Y;
    p.ldy = d.ldy;
    p.rows = d.rows;
    p.K = d.K;
    p.N = d.N;
    p.accumulate = d.accumulate != 0;
    p.drop_seed = d.drop_seed;
    p.drop_keep = d.drop_keep;
    p.drop_scale = d.drop_scale;
    p.res = d.res;
    p.ldres = d.ldres;
    p.Y2 = d.Y2;
    p.ldy2 = d.ldy2;
    p.binarize_a = d.binarize_a;
    p.row_inv = d.row_inv;
    p.b_row_count = d.b_row_count;
    p.b_scale = d.b_scale;
    p.a_drop_seed = d.a_drop_seed;
    p.a_drop_keep = d.a_drop_keep;
    p.a_drop_scale = d.a_drop_scale;
  }
  g.count = count;
  return row_gemm_group(g, as_stream(stream), "hgd_gemm_rows");
}

extern "C" size_t hgd_linear_backward_weight_workspace_size(int64_t n_rows, int32_t out_features,
                                                           int32_t in_features) {
  if (n_rows <= 0 || out_features <= 0 || in_features <= 0) return 0;
  hgd_gemm_tn_desc d{};
  d.rows = n_rows;
  d.M = out_features;
  d.N = in_features;
  d.colsum_A = reinterpret_cast<float*>(16);  // sized with the bias partials
  return hgd_gemm_tn_workspace_size(&d, 1);
}

extern "C" hgd_status hgd_linear_backward_weight(const float* dY, int64_t ldy,
                                                 const float* relu_out, int64_t ldr,
                                                 const float* X, int64_t ldx, int64_t n_rows,
                                                 int32_t out_features, int32_t in_features,
                                                 float* dW, float* db, void* workspace,
                                                 size_t workspace_bytes, void* stream) {
  hgd_gemm_tn_desc d{};
  d.A = dY;
  d.lda = ldy;
  d.relu_mask = relu_out;
  d.ldm = ldr;
  d.B = X;
  d.ldb = ldx;
  d.rows = n_rows;
  d.M = out_features;
  d.N = in_features;
  d.C = dW;
  d.colsum_A = db;
  return hgd_gemm_tn(&d, 1, workspace, workspace_bytes, stream);
}
