// Fused InfoNCE (contrastLoss, util/loss_torch.py:103-110):
//
//   p1 = normalize(E1[nodes] + 1e-8), p2 = normalize(E2[nodes] + 1e-8)      (F.normalize, eps 1e-12)
//   loss = -mean_b log( exp(<p1_b,p2_b>/τ) / (Σ_j exp(<p1_b,p2_j>/τ) + 1e-8) )
//
// The reference normalises the WHOLE [N, d] tables before gathering the B batch rows and
// materialises the [B, B] logits (plus their exp) for autograd. Here:
//   * k_nce_gather: one lane group per batch row gathers, shifts and normalises only the B rows
//     of both tables (and the positive logit <p1_b, p2_b>/τ, summed like torch.sum);
//   * k_nce_rowsum: the [B, B] exp-sum flash-style on the f32 MFMA (v_mfma_f32_16x16x4_f32):
//     each wave owns 16 rows of p1 (fragments in registers) and streams 16-column tiles of p2,
//     exponentiating the 16×16 logit tile in registers; the j range is split over S workgroups
//     whose partial row sums are added in a fixed order (deterministic, no atomics);
//   * the diagonal is kept apart: k_nce_rowsum sums the OFF-diagonal terms (off_b =
//     Σ_{j≠b} exp(s_bj/τ) + 1e-8) and leaves exp(s_bb/τ) for the finish, which forms
//     deno_b = off_b + exp(s_bb/τ) and keeps off_b beside it (deno holds [2, B]). The loss term
//     log(deno_b/nume_b) is then log1p((off_b + (e_bb − nume_b))/nume_b), and the diagonal
//     gradient weight −(1 − p_bb) is −off_b/deno_b: no cancellation of p_bb ≈ 1 against 1. That
//     case is HCCF's (HCCF.py:65-66 passes torch.unique(emb.long()), often a list of one or two
//     nodes: p_bb = e/(e + 1e-8) rounds to 1 in fp32, so e/deno − 1 is pure rounding noise and the
//     reference's own fp32 autograd returns noise there — we return the float64 value's digits);
//   * backward: G_bj = g·(exp(s_bj/τ)/deno_b − δ_bj)/(B·τ) is recomputed tile by tile, and
//     dP1 = G·P2, dP2 = Gᵀ·P1 run on the MFMA with the logit tile's accumulator registers used
//     directly as the next MFMA's A operand (rows of the tile on the lane, its columns in the
//     4 registers = the k index, in a permuted order the B operand follows); the split-j partials
//     are summed in order and the F.normalize backward (dx = (dp − p<p,dp>)/‖x‖) is fused into
//     that final pass. The scatter into the [N, d] table gradients is left to the caller.
#include <algorithm>

#include "device_util.h"
#include "hgd_internal.h"

namespace hgd {
namespace {

constexpr float kShift = 1e-8f;   // embeds + 1e-8 (loss_torch.py:104-105)
constexpr float kNormEps = 1e-12f;  // F.normalize eps
constexpr float kDenoEps = 1e-8f;   // ... .sum(-1) + 1e-8 (loss_torch.py:109)

// exp(s/τ) as 2^(s·k2) with k2 = log2(e)/τ rounded once on the host: the bare v_exp_f32 (about
// 1 ulp) instead of expf's 12-instruction range reduction. The extra error is the rounding of
// s·k2, |s·k2|·2^-24 relative (3e-7 at τ = 0.05, |s| ≤ 1): far inside the 1e-5 bound, and the
// forward sums and the backward's recomputed weights use the same formula. Results below 2^-126
// flush to 0 (a logit 87·τ below the row's: no weight at fp32 resolution of the sum anyway).
__device__ __forceinline__ float exp2_raw(float x) { return __builtin_amdgcn_exp2f(x); }

inline float exp2_scale(float temp) {
  return static_cast<float>(1.4426950408889634 / static_cast<double>(temp));
}

// One InfoNCE term's operands. Up to kMaxTerms terms run as ONE launch per kernel (HCCF's user
// and item terms of every layer, HCCF.py:62-67): blocks [start[i], start[i+1]) along x take p[i].
struct NceProb {
  const float* E1;
  int64_t ld1;
  const float* E2;
  int64_t ld2;
  int64_t n_rows;
  const int64_t* nodes;
  int64_t B;          // capacity (strides, grid)
  const int64_t* Bp;  // live count on the device, or NULL (= B)
  float* P1;
  float* P2;
  float* inv1;
  float* inv2;
  float* pos_logit;
  float* deno;
  float* loss;
  float* partial;  // forward [S, B]
  float* part1;    // backward [S, B, d] (dP1 side)
  float* part2;    // backward [S, B, d] (dP2 side)
  int64_t per_slice;
  int64_t S_used;
  float* dX1;  // backward outputs: compact [B, d] rows, or scatter into dE
  float* dX2;
  float* dE1;
  int64_t ldE1;
  float* dE2;
  int64_t ldE2;
};

constexpr int kMaxTerms = 8;

struct NceGroup {
  NceProb p[kMaxTerms];
  int32_t count;
  int32_t start[kMaxTerms];  // first x-block of each term
};

__device__ __forceinline__ NceProb pick(const NceGroup& g, int64_t& bx) {
  int i = 0;
#pragma unroll
  for (int k = 1; k < kMaxTerms; ++k)
    if (k < g.count && bx >= g.start[k]) i = k;
  bx -= g.start[i];
  return g.p[i];
}

// ---- gather + normalise: one group of G = d/4 lanes per batch row ----
template <int G>
__global__ __launch_bounds__(256) void k_nce_gather(NceGroup grp, int32_t d, float inv_temp) {
  constexpr int GPB = 256 / G;
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  int64_t bx = blockIdx.x;
  const NceProb p = pick(grp, bx);
  const int64_t b = bx * GPB + g;
  if (b >= p.B) return;
  if (p.Bp && b >= *p.Bp) return;  // a capacity row past the device-side count: never read
  // torch indexing semantics: negative ids count from the end (the reference passes
  // torch.unique(emb.long()), HCCF.py:65-66, which yields -1 / 0 / 1); out-of-range ids are
  // rejected by the caller — clamped here only so that no load leaves the table
  int64_t node = p.nodes[b];
  if (node < 0) node += p.n_rows;
  node = node < 0 ? 0 : (node >= p.n_rows ? p.n_rows - 1 : node);
  const int c0 = 4 * l;
  const bool ok = c0 < d;
  f32x4 x1 = {0.f, 0.f, 0.f, 0.f}, x2 = {0.f, 0.f, 0.f, 0.f};
  if (ok) {
    x1 = *reinterpret_cast<const f32x4*>(p.E1 + node * p.ld1 + c0) + kShift;
    x2 = *reinterpret_cast<const f32x4*>(p.E2 + node * p.ld2 + c0) + kShift;
  }
  const float n1 = sqrtf(group_sum<G>(x1.x * x1.x + x1.y * x1.y + x1.z * x1.z + x1.w * x1.w));
  const float n2 = sqrtf(group_sum<G>(x2.x * x2.x + x2.y * x2.y + x2.z * x2.z + x2.w * x2.w));
  const float r1 = 1.f / fmaxf(n1, kNormEps);
  const float r2 = 1.f / fmaxf(n2, kNormEps);
  const f32x4 p1 = x1 * r1, p2 = x2 * r2;
  const float dot = group_sum<G>(p1.x * p2.x + p1.y * p2.y + p1.z * p2.z + p1.w * p2.w);
  if (ok) {
    *reinterpret_cast<f32x4*>(p.P1 + b * d + c0) = p1;
    *reinterpret_cast<f32x4*>(p.P2 + b * d + c0) = p2;
  }
  if (l == 0) {
    p.inv1[b] = r1;
    p.inv2[b] = r2;
    p.pos_logit[b] = dot * inv_temp;
  }
}

// Fragments of rows [r0, r0+16) of a [B, d] matrix as float4 loads: lane l holds
// M[r0 + (l&15)][4(l>>4) + 16q' .. +3] for q' < d/16, i.e. MFMA step (q', c) multiplies
// k = 4(l>>4) + 16q' + c — a fixed permutation of k that every operand loaded this way shares.
// Rows past B are clamped (their contributions are masked by the callers).
template <int DQ>
__device__ __forceinline__ void load_frag4(const float* M, int64_t B, int d, int64_t r0, int lane,
                                           f32x4 (&f)[DQ / 4]) {
  int64_t r = r0 + (lane & 15);
  r = r < B ? r : B - 1;
  const float* row = M + r * d + 4 * (lane >> 4);
#pragma unroll
  for (int q = 0; q < DQ / 4; ++q) f[q] = *reinterpret_cast<const f32x4*>(row + 16 * q);
}

// ---- shared staging of the streamed rows ----
// The four waves of a workgroup own different 16-row blocks but stream the SAME rows of the other
// matrix, so those rows go through LDS once per workgroup (a quarter of the L2 traffic of per-wave
// loads, and no register ping-pong: the double buffer is in LDS). A stage is KT rows, loaded
// cooperatively as float4s into registers while the previous stage is consumed, then written to
// the other LDS buffer behind one barrier. Rows are padded by 4 floats, so the 16 lanes that read
// 16 different rows at one column (a fragment load) hit 16 different bank quads.
constexpr int kStageRows = 32;

template <int DQ>
struct Stage {
  static constexpr int D = 4 * DQ;
  static constexpr int LDR = D + 4;                       // padded row (floats)
  static constexpr int PER = (kStageRows * DQ + 255) / 256;  // float4s per thread per stage
};

template <int DQ>
__device__ __forceinline__ void stage_load(const float* M, int64_t Be, int64_t k0,
                                           f32x4 (&v)[Stage<DQ>::PER]) {
#pragma unroll
  for (int i = 0; i < Stage<DQ>::PER; ++i) {
    const int e = threadIdx.x + 256 * i;
    int64_t row = k0 + e / DQ;
    row = row < Be ? row : Be - 1;  // rows past the live count: clamped, masked when consumed
    if (e < kStageRows * DQ) v[i] = ld4(M + row * (4 * DQ) + 4 * (e % DQ));
  }
}

template <int DQ>
__device__ __forceinline__ void stage_store(float* s, const f32x4 (&v)[Stage<DQ>::PER]) {
#pragma unroll
  for (int i = 0; i < Stage<DQ>::PER; ++i) {
    const int e = threadIdx.x + 256 * i;
    if (e < kStageRows * DQ)
      *reinterpret_cast<f32x4*>(s + (e / DQ) * Stage<DQ>::LDR + 4 * (e % DQ)) = v[i];
  }
}

// Fragment of rows [r0, r0+16) of a staged tile, in load_frag4's k order.
template <int DQ>
__device__ __forceinline__ void lds_frag4(const float* s, int r0, int lane, f32x4 (&f)[DQ / 4]) {
  const float* row = s + (r0 + (lane & 15)) * Stage<DQ>::LDR + 4 * (lane >> 4);
#pragma unroll
  for (int q = 0; q < DQ / 4; ++q) f[q] = *reinterpret_cast<const f32x4*>(row + 16 * q);
}

// ---- forward exp-sums: partial[s][b] = Σ_{j in slice s} exp(<p1_b, p2_j>/τ) ----
// A wave owns 16 rows of p1 (fragments in registers); the slice's p2 rows stream through LDS in
// 32-row stages shared by the workgroup's four waves.
template <int DQ>  // d = 4·DQ
__global__ __launch_bounds__(256) void k_nce_rowsum(NceGroup grp, float k2) {
  using St = Stage<DQ>;
  constexpr int Q4 = DQ / 4;
  __shared__ float sm[2][kStageRows * St::LDR];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  int64_t bx = blockIdx.x;
  const NceProb p = pick(grp, bx);
  if (static_cast<int64_t>(blockIdx.y) >= p.S_used) return;  // uniform over the workgroup
  const float* __restrict__ P1 = p.P1;
  const float* __restrict__ P2 = p.P2;
  const int64_t B = p.B;
  const int64_t Be = p.Bp ? *p.Bp : B;  // live rows (B is the capacity: strides, clamps)
  const int64_t blk0 = bx * 64;
  if (blk0 >= Be) return;  // uniform over the workgroup
  const int64_t b0 = blk0 + 16 * wave;
  const int d = 4 * DQ;
  f32x4 a[Q4];
  load_frag4<DQ>(P1, Be, d, b0 < Be ? b0 : blk0, lane, a);  // a wave past the end: dummy rows
  const int64_t j_begin = static_cast<int64_t>(blockIdx.y) * p.per_slice;
  const int64_t j_end = min(Be, j_begin + p.per_slice);
  float psum[4] = {0.f, 0.f, 0.f, 0.f};
  f32x4 v[St::PER];
  stage_load<DQ>(P2, Be, j_begin, v);
  stage_store<DQ>(sm[0], v);
  __syncthreads();
  int buf = 0;
  for (int64_t j0 = j_begin; j0 < j_end; j0 += kStageRows) {
    const bool more = j0 + kStageRows < j_end;
    if (more) stage_load<DQ>(P2, Be, j0 + kStageRows, v);
#pragma unroll
    for (int t = 0; t < kStageRows / 16; ++t) {
      f32x4 f[Q4];
      lds_frag4<DQ>(sm[buf], 16 * t, lane, f);
      f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < Q4; ++q)
#pragma unroll
        for (int c = 0; c < 4; ++c) s = mfma4(a[q][c], f[q][c], s);
      // s[r] = <p1_{b0 + 4(l>>4) + r}, p2_{j0 + 16t + (l&15)}>
      const int64_t j = j0 + 16 * t + (lane & 15);
      const bool jok = j < j_end;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t b = b0 + 4 * (lane >> 4) + r;
        const float e = exp2_raw(s[r] * k2);
        if (j == b) {  // the diagonal: exactly one lane of the grid; kept apart for the finish
          if (jok && b < Be) p.deno[b] = e;
        } else {
          psum[r] += jok ? e : 0.f;
        }
      }
    }
    if (more) stage_store<DQ>(sm[buf ^ 1], v);
    __syncthreads();
    buf ^= 1;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) psum[r] = group_sum<16>(psum[r]);
  if ((lane & 15) == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t b = b0 + 4 * (lane >> 4) + r;
      if (b < Be) p.partial[static_cast<int64_t>(blockIdx.y) * B + b] = psum[r];
    }
  }
}

// ---- finish: deno_b, loss = -(1/B) Σ_b log(exp(pos_b) / deno_b), fixed-order reductions ----
// One workgroup; each thread's rows are summed over the S slice partials in slice order, eight
// independent loads at a time (a serial chain of S dependent loads per row was 19 µs at B = 4096).
__global__ __launch_bounds__(1024) void k_nce_finish(NceGroup grp) {
  const NceProb& p = grp.p[blockIdx.x];  // one workgroup per term
  const float* __restrict__ partial = p.partial;
  const float* __restrict__ pos_logit = p.pos_logit;
  const int64_t S = p.S_used, B = p.B;
  float* deno = p.deno;
  __shared__ float red[1024];
  const int64_t Be = p.Bp ? *p.Bp : B;
  float acc = 0.f;
  for (int64_t b = threadIdx.x; b < Be; b += 1024) {
    float den = 0.f;
    int64_t s = 0;
    for (; s + 8 <= S; s += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = partial[(s + u) * B + b];
#pragma unroll
      for (int u = 0; u < 8; ++u) den += v[u];
    }
    for (; s < S; ++s) den += partial[s * B + b];
    const float off = den + kDenoEps;  // Σ_{j≠b} exp(s_bj/τ) + 1e-8
    const float e_bb = deno[b];        // exp(s_bb/τ), left by k_nce_rowsum
    const float nume = expf(pos_logit[b]);
    deno[b] = off + e_bb;
    deno[B + b] = off;
    // log(nume / deno) = −log1p((deno − nume)/nume), deno − nume = off + (e_bb − nume): the two
    // exps are the same logit rounded two ways, so their difference is exact-ish (Sterbenz)
    acc -= log1pf((off + (e_bb - nume)) / nume);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 512; w >= 1; w >>= 1) {
    if (static_cast<int>(threadIdx.x) < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *p.loss = -red[0] / static_cast<float>(Be);
}

// ---- backward partials ----
// ROWS = true : part[s][b][:] = Σ_{j in slice s} G_bj p2_j       (dP1)
// ROWS = false: part[s][j][:] = Σ_{b in slice s} G_bj p1_b       (dP2)
// with G_bj = coef·(exp(s_bj/τ)/deno_b − δ_bj), coef = g/(B·τ); the diagonal as −coef·off_b/deno_b.
// The "other" rows of the slice stream through LDS in 32-row stages shared by the workgroup's
// four waves (with their denominators when those index the other rows); each 16-row tile is read
// twice from the stage: as logit fragments (row on the lane) and, transposed, as the B operand of
// the accumulation (feature on the lane) — the LDS read replaces the per-lane strided scalar
// loads of that operand.
template <int DQ, bool ROWS>
__global__ __launch_bounds__(256) void k_nce_bwd(NceGroup grp, float k2,
                                                 const float* __restrict__ grad, float temp) {
  using St = Stage<DQ>;
  constexpr int Q4 = DQ / 4;
  __shared__ float sm[2][kStageRows * St::LDR];
  __shared__ float sinv[2][kStageRows];  // 1/deno of the staged other rows (ROWS = false)
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int i16 = lane & 15;
  const int h = lane >> 4;
  const int d = 4 * DQ;
  int64_t bx = blockIdx.x;
  const NceProb p = pick(grp, bx);
  if (static_cast<int64_t>(blockIdx.y) >= p.S_used) return;  // uniform over the workgroup
  const float* __restrict__ P1 = p.P1;
  const float* __restrict__ P2 = p.P2;
  const float* __restrict__ deno = p.deno;
  const int64_t B = p.B;
  float* part = ROWS ? p.part1 : p.part2;
  const int64_t Be = p.Bp ? *p.Bp : B;  // live rows (B is the capacity: strides, clamps)
  const int64_t blk0 = bx * 64;
  if (blk0 >= Be) return;  // uniform over the workgroup
  // upstream dL/dloss and the 1/(B·τ) of the mean: device values, no host sync
  const float coef = grad[0] / (static_cast<float>(Be) * temp);
  // "own" rows: b (ROWS) or j (!ROWS); "other" rows are streamed
  const float* own_m = ROWS ? P1 : P2;
  const float* oth_m = ROWS ? P2 : P1;
  const int64_t o0 = blk0 + 16 * wave;
  f32x4 own[Q4];
  load_frag4<DQ>(own_m, Be, d, o0 < Be ? o0 : blk0, lane, own);  // rows clamped to live ones
  const int64_t o_lane = o0 + i16;  // own row of this lane in the logit tile below
  float inv_own = 1.f;
  if (ROWS) inv_own = 1.f / deno[o_lane < Be ? o_lane : Be - 1];
  // the diagonal weight −(1 − p_bb) = −off_b/deno_b of this lane's own row (off_b: deno[B + b])
  const float off_own = deno[B + (o_lane < Be ? o_lane : Be - 1)];
  const int64_t k_begin = static_cast<int64_t>(blockIdx.y) * p.per_slice;
  const int64_t k_end = min(Be, k_begin + p.per_slice);
  f32x4 acc[DQ / 4];
#pragma unroll
  for (int t = 0; t < DQ / 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto load_inv = [&](int64_t k0) -> float {
    if (ROWS || threadIdx.x >= kStageRows) return 0.f;
    int64_t k = k0 + threadIdx.x;
    k = k < Be ? k : Be - 1;
    return 1.f / deno[k];
  };
  f32x4 v[St::PER];
  stage_load<DQ>(oth_m, Be, k_begin, v);
  float vinv = load_inv(k_begin);
  stage_store<DQ>(sm[0], v);
  if (!ROWS && threadIdx.x < kStageRows) sinv[0][threadIdx.x] = vinv;
  __syncthreads();
  int buf = 0;
  for (int64_t k0 = k_begin; k0 < k_end; k0 += kStageRows) {
    const bool more = k0 + kStageRows < k_end;
    if (more) {
      stage_load<DQ>(oth_m, Be, k0 + kStageRows, v);
      vinv = load_inv(k0 + kStageRows);
    }
    const float* s_tile = sm[buf];
#pragma unroll
    for (int u = 0; u < kStageRows / 16; ++u) {
      const int64_t kt = k0 + 16 * u;
      // logit tile with the OTHER index on the output rows:
      // s[r] = <oth_{kt + 4(l>>4) + r}, own_{o0 + (l&15)}>
      f32x4 of[Q4];
      lds_frag4<DQ>(s_tile, 16 * u, lane, of);
      f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < Q4; ++q)
#pragma unroll
        for (int c = 0; c < 4; ++c) s = mfma4(of[q][c], own[q][c], s);
      float gk[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t k = kt + 4 * h + r;  // other index of register r
        const float e = exp2_raw(s[r] * k2);
        const float inv = ROWS ? inv_own : sinv[buf][16 * u + 4 * h + r];
        const float w = (k == o_lane) ? -off_own * inv : e * inv;
        gk[r] = (k < k_end && o_lane < Be) ? coef * w : 0.f;
      }
      // acc[own row][n] += Σ_k G[own][k]·oth_k[n]: A operand = gk (own row on the lane, k-step
      // r covers other rows {4(l>>4) + r}), B operand = those rows' features, read transposed
      // from the stage: bv = oth[kt + 4(l>>4) + r][16t + (l&15)]
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float* brow = s_tile + (16 * u + 4 * h + r) * St::LDR + i16;
#pragma unroll
        for (int t = 0; t < DQ / 4; ++t) acc[t] = mfma4(gk[r], brow[16 * t], acc[t]);
      }
    }
    if (more) {
      stage_store<DQ>(sm[buf ^ 1], v);
      if (!ROWS && threadIdx.x < kStageRows) sinv[buf ^ 1][threadIdx.x] = vinv;
    }
    __syncthreads();
    buf ^= 1;
  }
  if (o0 >= Be) return;
  // acc[t] reg r: own row o0 + 4(l>>4) + r, feature 16t + (l&15)
#pragma unroll
  for (int t = 0; t < DQ / 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t o = o0 + 4 * h + r;
      if (o < Be) part[(static_cast<int64_t>(blockIdx.y) * B + o) * d + 16 * t + i16] =
          acc[t][r];
    }
}

// ---- sum the split partials in order and apply the F.normalize backward per row ----
template <int G, bool SIDE1>
__global__ __launch_bounds__(256) void k_nce_norm_bwd(NceGroup grp, int32_t d) {
  constexpr int GPB = 256 / G;
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  int64_t bx = blockIdx.x;
  const NceProb q = pick(grp, bx);
  const float* __restrict__ part = SIDE1 ? q.part1 : q.part2;
  const float* __restrict__ P = SIDE1 ? q.P1 : q.P2;
  const float* __restrict__ inv = SIDE1 ? q.inv1 : q.inv2;
  float* dX = SIDE1 ? q.dX1 : q.dX2;
  float* dE = SIDE1 ? q.dE1 : q.dE2;
  const int64_t ldE = SIDE1 ? q.ldE1 : q.ldE2;
  if (!dX && !dE) return;  // this term does not want this side (uniform)
  const int64_t S = q.S_used, B = q.B, n_rows = q.n_rows;
  const int64_t b = bx * GPB + g;
  if (b >= B) return;
  const int c0 = 4 * l;
  const bool ok = c0 < d;
  if (q.Bp && b >= *q.Bp) {  // capacity row: a zero gradient row, or nothing to scatter
    if (ok && dX) *reinterpret_cast<f32x4*>(dX + b * d + c0) = f32x4{0.f, 0.f, 0.f, 0.f};
    return;
  }
  f32x4 dp = {0.f, 0.f, 0.f, 0.f}, p = {0.f, 0.f, 0.f, 0.f};
  if (ok) {
    for (int64_t s = 0; s < S; ++s) dp += *reinterpret_cast<const f32x4*>(part + (s * B + b) * d + c0);
    p = *reinterpret_cast<const f32x4*>(P + b * d + c0);
  }
  const float dot = group_sum<G>(p.x * dp.x + p.y * dp.y + p.z * dp.z + p.w * dp.w);
  const float r = inv[b];
  // F.normalize backward: x / max(‖x‖, eps); when ‖x‖ <= eps the op is x·(1/eps), linear
  const bool clamped = r >= 1.f / kNormEps;
  const f32x4 dx = clamped ? dp * r : (dp - p * dot) * r;
  if (!ok) return;
  if (dE) {
    // scatter-add into the [n_rows, d] table gradient at this batch row's node (torch indexing:
    // negative ids wrap). At most two batch rows meet on one table row (x and x − n), and a sum
    // of two terms onto 0 is order-independent, so the atomics stay deterministic.
    int64_t node = q.nodes[b];
    if (node < 0) node += n_rows;
    node = node < 0 ? 0 : (node >= n_rows ? n_rows - 1 : node);
    float* row = dE + node * ldE + c0;
    atomicAdd(row + 0, dx.x);
    atomicAdd(row + 1, dx.y);
    atomicAdd(row + 2, dx.z);
    atomicAdd(row + 3, dx.w);
  } else {
    *reinterpret_cast<f32x4*>(dX + b * d + c0) = dx;
  }
}

// lanes per row for the row kernels: the next power of two ≥ d/4 (each lane holds 4 columns)
int group_for(int d) {
  int g = 4;
  while (g < d / 4) g <<= 1;
  return g;
}

int64_t slices_for(int64_t B) {
  // ≈ 4 workgroups per CU over the (B/64) × S grid, each slice at least 128 columns
  const int64_t row_blocks = (B + 63) / 64;
  int64_t s = (1024 + row_blocks - 1) / row_blocks;
  const int64_t max_s = (B + 127) / 128;
  if (s > max_s) s = max_s;
  return s < 1 ? 1 : s;
}

int64_t per_slice(int64_t B, int64_t S) {
  int64_t p = (B + S - 1) / S;
  return (p + 63) / 64 * 64;  // whole 64-row super-tiles
}

}  // namespace
}  // namespace hgd

extern "C" size_t hgd_infonce_workspace_size(int64_t batch, int32_t d) {
  if (batch <= 0 || d <= 0) return 0;
  const size_t S = static_cast<size_t>(hgd::slices_for(batch));
  const size_t B = static_cast<size_t>(batch);
  // forward partial sums [S, B]; backward partials 2 × [S, B, d]
  return hgd::align_up(S * B * 4) + 2 * hgd::align_up(S * B * static_cast<size_t>(d) * 4);
}

namespace hgd {
namespace {

// Checks one term and fills its problem descriptor (workspace partition, slice plan).
hgd_status prepare(const hgd_infonce_term& t, int32_t d, bool backward, NceProb* p,
                   const char* fn) {
  HGD_REQUIRE(t.capacity > 0, "%s: empty batch", fn);
  HGD_REQUIRE(d % 16 == 0 && d >= 16 && d <= 256, "%s: d = %d must be a multiple of 16 in [16, 256]",
              fn, d);
  const size_t need = hgd_infonce_workspace_size(t.capacity, d);
  if (t.workspace_bytes < need || !t.workspace)
    return fail(HGD_ERR_WORKSPACE, "%s: workspace %zu < required %zu", fn, t.workspace_bytes,
                need);
  HGD_REQUIRE(t.P1 && t.P2 && t.inv_norm1 && t.inv_norm2 && t.deno, "%s: null pointer", fn);
  if (!backward) {
    HGD_REQUIRE(t.n_rows > 0, "%s: empty table", fn);
    HGD_REQUIRE(t.ld1 >= d && t.ld2 >= d && t.ld1 % 4 == 0 && t.ld2 % 4 == 0,
                "%s: leading dimensions must be >= d and multiples of 4", fn);
    HGD_REQUIRE(t.E1 && t.E2 && t.nodes && t.pos_logit && t.loss, "%s: null pointer", fn);
    HGD_REQUIRE(reinterpret_cast<uintptr_t>(t.E1) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(t.E2) % 16 == 0,
                "%s: tables must be 16-byte aligned", fn);
  } else {
    const bool side1 = t.dX1 || t.dE1, side2 = t.dX2 || t.dE2;
    HGD_REQUIRE(side1 || side2, "%s: no output", fn);
    HGD_REQUIRE(!(t.dE1 || t.dE2) || (t.nodes && t.n_rows > 0 && (!t.dE1 || t.ldE1 >= d) &&
                                      (!t.dE2 || t.ldE2 >= d)),
                "%s: a table scatter needs nodes, n_rows and ld >= d", fn);
  }
  const int64_t B = t.capacity;
  const int64_t S = slices_for(B);
  const int64_t ps = per_slice(B, S);
  NceProb& q = *p;
  q = NceProb{};
  q.E1 = t.E1; q.ld1 = t.ld1; q.E2 = t.E2; q.ld2 = t.ld2; q.n_rows = t.n_rows;
  q.nodes = t.nodes; q.B = B; q.Bp = t.batch_count;
  q.P1 = t.P1; q.P2 = t.P2; q.inv1 = t.inv_norm1; q.inv2 = t.inv_norm2;
  q.pos_logit = t.pos_logit; q.deno = t.deno; q.loss = t.loss;
  char* ws = static_cast<char*>(t.workspace);
  const size_t off = align_up(static_cast<size_t>(S) * B * 4);
  q.partial = reinterpret_cast<float*>(ws);
  q.part1 = reinterpret_cast<float*>(ws + off);
  q.part2 = reinterpret_cast<float*>(ws + off + align_up(static_cast<size_t>(S) * B * d * 4));
  q.per_slice = ps;
  q.S_used = (B + ps - 1) / ps;
  q.dX1 = t.dX1; q.dX2 = t.dX2; q.dE1 = t.dE1; q.ldE1 = t.ldE1; q.dE2 = t.dE2; q.ldE2 = t.ldE2;
  return HGD_OK;
}

// x-blocks of each term for a kernel with `rows_per_block` batch rows per workgroup
NceGroup group_of(const NceProb* p, int count, int64_t rows_per_block, unsigned* grid_x) {
  NceGroup g{};
  g.count = count;
  int64_t total = 0;
  for (int i = 0; i < count; ++i) {
    g.p[i] = p[i];
    g.start[i] = static_cast<int32_t>(total);
    total += (p[i].B + rows_per_block - 1) / rows_per_block;
  }
  *grid_x = static_cast<unsigned>(total);
  return g;
}

hgd_status infonce_forward(const hgd_infonce_term* terms, int count, int32_t d, float temp,
                           hipStream_t st, const char* fn) {
  HGD_REQUIRE(terms && count >= 1 && count <= kMaxTerms, "%s: 1 to %d terms", fn, kMaxTerms);
  HGD_REQUIRE(temp > 0.f, "%s: temperature must be > 0", fn);
  NceProb p[kMaxTerms];
  int64_t s_max = 1;
  for (int i = 0; i < count; ++i) {
    const hgd_status c = prepare(terms[i], d, false, &p[i], fn);
    if (c != HGD_OK) return c;
    s_max = std::max<int64_t>(s_max, p[i].S_used);
  }
  const float inv_temp = 1.f / temp;
  const float k2 = exp2_scale(temp);
  const int G = group_for(d);
  unsigned gx = 0;
  NceGroup gg = group_of(p, count, 256 / G, &gx);
  switch (G) {
    case 4: hipLaunchKernelGGL((k_nce_gather<4>), dim3(gx), dim3(256), 0, st, gg, d, inv_temp); break;
    case 8: hipLaunchKernelGGL((k_nce_gather<8>), dim3(gx), dim3(256), 0, st, gg, d, inv_temp); break;
    case 16: hipLaunchKernelGGL((k_nce_gather<16>), dim3(gx), dim3(256), 0, st, gg, d, inv_temp); break;
    case 32: hipLaunchKernelGGL((k_nce_gather<32>), dim3(gx), dim3(256), 0, st, gg, d, inv_temp); break;
    default: hipLaunchKernelGGL((k_nce_gather<64>), dim3(gx), dim3(256), 0, st, gg, d, inv_temp); break;
  }
  hgd_status s = check_launch("hgd_infonce forward gather");
  if (s != HGD_OK) return s;
  NceGroup gr = group_of(p, count, 64, &gx);
  const dim3 grid(gx, static_cast<unsigned>(s_max));
  switch (d / 4) {
#define HGD_CASE(DQ)                                                                       \
    case DQ:                                                                               \
      hipLaunchKernelGGL((k_nce_rowsum<DQ>), grid, dim3(256), 0, st, gr, k2);              \
      break;
    HGD_CASE(4) HGD_CASE(8) HGD_CASE(12) HGD_CASE(16) HGD_CASE(20) HGD_CASE(24) HGD_CASE(28)
    HGD_CASE(32) HGD_CASE(36) HGD_CASE(40) HGD_CASE(44) HGD_CASE(48) HGD_CASE(52) HGD_CASE(56)
    HGD_CASE(60) HGD_CASE(64)
#undef HGD_CASE
    default: return fail(HGD_ERR_UNSUPPORTED, "%s: d = %d", fn, d);
  }
  s = check_launch("hgd_infonce forward rowsum");
  if (s != HGD_OK) return s;
  hipLaunchKernelGGL(k_nce_finish, dim3(count), dim3(1024), 0, st, gr);
  return check_launch("hgd_infonce forward finish");
}

hgd_status infonce_backward(const hgd_infonce_term* terms, int count, int32_t d, float temp,
                            const float* grad_loss, hipStream_t st, const char* fn) {
  HGD_REQUIRE(terms && count >= 1 && count <= kMaxTerms, "%s: 1 to %d terms", fn, kMaxTerms);
  HGD_REQUIRE(temp > 0.f, "%s: temperature must be > 0", fn);
  HGD_REQUIRE(grad_loss, "%s: null grad_loss", fn);
  NceProb p[kMaxTerms];
  int64_t s_max = 1;
  bool side1 = false, side2 = false;
  for (int i = 0; i < count; ++i) {
    const hgd_status c = prepare(terms[i], d, true, &p[i], fn);
    if (c != HGD_OK) return c;
    s_max = std::max<int64_t>(s_max, p[i].S_used);
    side1 = side1 || p[i].dX1 || p[i].dE1;
    side2 = side2 || p[i].dX2 || p[i].dE2;
  }
  // a side is computed for every term of the launch when any term wants it (its partials go
  // to that term's workspace; the norm pass skips a term without that side's output)
  const float k2 = exp2_scale(temp);
  unsigned gx = 0;
  NceGroup gr = group_of(p, count, 64, &gx);
  const dim3 grid(gx, static_cast<unsigned>(s_max));
  switch (d / 4) {
#define HGD_CASE(DQ)                                                                           \
    case DQ:                                                                                   \
      if (side1)                                                                               \
        hipLaunchKernelGGL((k_nce_bwd<DQ, true>), grid, dim3(256), 0, st, gr, k2, grad_loss,   \
                           temp);                                                              \
      if (side2)                                                                               \
        hipLaunchKernelGGL((k_nce_bwd<DQ, false>), grid, dim3(256), 0, st, gr, k2, grad_loss,  \
                           temp);                                                              \
      break;
    HGD_CASE(4) HGD_CASE(8) HGD_CASE(12) HGD_CASE(16) HGD_CASE(20) HGD_CASE(24) HGD_CASE(28)
    HGD_CASE(32) HGD_CASE(36) HGD_CASE(40) HGD_CASE(44) HGD_CASE(48) HGD_CASE(52) HGD_CASE(56)
    HGD_CASE(60) HGD_CASE(64)
#undef HGD_CASE
    default: return fail(HGD_ERR_UNSUPPORTED, "%s: d = %d", fn, d);
  }
  hgd_status s = check_launch("hgd_infonce backward partials");
  if (s != HGD_OK) return s;
  const int G = group_for(d);
  NceGroup gn = group_of(p, count, 256 / G, &gx);
  switch (G) {
#define HGD_CASE(GG)                                                                         \
    case GG:                                                                                 \
      if (side1)                                                                             \
        hipLaunchKernelGGL((k_nce_norm_bwd<GG, true>), dim3(gx), dim3(256), 0, st, gn, d);  \
      if (side2)                                                                             \
        hipLaunchKernelGGL((k_nce_norm_bwd<GG, false>), dim3(gx), dim3(256), 0, st, gn, d); \
      break;
    HGD_CASE(4) HGD_CASE(8) HGD_CASE(16) HGD_CASE(32) HGD_CASE(64)
#undef HGD_CASE
    default: return fail(HGD_ERR_UNSUPPORTED, "%s: group %d", fn, G);
  }
  return check_launch("hgd_infonce backward norm");
}

hgd_infonce_term term_of(const float* E1, int64_t ld1, const float* E2, int64_t ld2,
                         int64_t n_rows, const int64_t* nodes, int64_t capacity,
                         const int64_t* batch_count, float* P1, float* P2, float* inv1,
                         float* inv2, float* pos_logit, float* deno, float* loss, void* ws,
                         size_t wsb) {
  hgd_infonce_term t{};
  t.E1 = E1; t.ld1 = ld1; t.E2 = E2; t.ld2 = ld2; t.n_rows = n_rows; t.nodes = nodes;
  t.capacity = capacity; t.batch_count = batch_count; t.P1 = P1; t.P2 = P2;
  t.inv_norm1 = inv1; t.inv_norm2 = inv2; t.pos_logit = pos_logit; t.deno = deno; t.loss = loss;
  t.workspace = ws; t.workspace_bytes = wsb;
  return t;
}

}  // namespace
}  // namespace hgd

extern "C" hgd_status hgd_infonce_forward(const float* E1, int64_t ld1, const float* E2,
                                          int64_t ld2, int64_t n_rows, const int64_t* nodes,
                                          int64_t batch, int32_t d, float temp, float* P1,
                                          float* P2, float* inv_norm1, float* inv_norm2,
                                          float* pos_logit, float* deno, float* loss,
                                          void* workspace, size_t workspace_bytes,
                                          void* stream) {
  hgd::clear_error();
  const hgd_infonce_term t = hgd::term_of(E1, ld1, E2, ld2, n_rows, nodes, batch, nullptr, P1,
                                          P2, inv_norm1, inv_norm2, pos_logit, deno, loss,
                                          workspace, workspace_bytes);
  return hgd::infonce_forward(&t, 1, d, temp, hgd::as_stream(stream), "hgd_infonce_forward");
}

extern "C" hgd_status hgd_infonce_forward_n(const float* E1, int64_t ld1, const float* E2,
                                            int64_t ld2, int64_t n_rows, const int64_t* nodes,
                                            int64_t capacity, const int64_t* batch_count,
                                            int32_t d, float temp, float* P1, float* P2,
                                            float* inv_norm1, float* inv_norm2, float* pos_logit,
                                            float* deno, float* loss, void* workspace,
                                            size_t workspace_bytes, void* stream) {
  hgd::clear_error();
  HGD_REQUIRE(batch_count, "hgd_infonce_forward_n: null batch_count");
  const hgd_infonce_term t = hgd::term_of(E1, ld1, E2, ld2, n_rows, nodes, capacity, batch_count,
                                          P1, P2, inv_norm1, inv_norm2, pos_logit, deno, loss,
                                          workspace, workspace_bytes);
  return hgd::infonce_forward(&t, 1, d, temp, hgd::as_stream(stream), "hgd_infonce_forward_n");
}

extern "C" hgd_status hgd_infonce_backward(const float* P1, const float* P2,
                                           const float* inv_norm1, const float* inv_norm2,
                                           const float* deno, int64_t batch, int32_t d,
                                           float temp, const float* grad_loss, float* dX1,
                                           float* dX2, void* workspace, size_t workspace_bytes,
                                           void* stream) {
  hgd::clear_error();
  HGD_REQUIRE(dX1 && dX2, "hgd_infonce_backward: null dX1/dX2");
  hgd_infonce_term t = hgd::term_of(nullptr, 0, nullptr, 0, 0, nullptr, batch, nullptr,
                                    const_cast<float*>(P1), const_cast<float*>(P2),
                                    const_cast<float*>(inv_norm1), const_cast<float*>(inv_norm2),
                                    nullptr, const_cast<float*>(deno), nullptr, workspace,
                                    workspace_bytes);
  t.dX1 = dX1;
  t.dX2 = dX2;
  return hgd::infonce_backward(&t, 1, d, temp, grad_loss, hgd::as_stream(stream),
                               "hgd_infonce_backward");
}

extern "C" hgd_status hgd_infonce_backward_n(const float* P1, const float* P2,
                                             const float* inv_norm1, const float* inv_norm2,
                                             const float* deno, int64_t capacity,
                                             const int64_t* batch_count, int32_t d, float temp,
                                             const float* grad_loss, const int64_t* nodes,
                                             int64_t n_rows, float* dE1, int64_t ldE1,
                                             float* dE2, int64_t ldE2, void* workspace,
                                             size_t workspace_bytes, void* stream) {
  hgd::clear_error();
  HGD_REQUIRE(batch_count, "hgd_infonce_backward_n: null batch_count");
  hgd_infonce_term t = hgd::term_of(nullptr, 0, nullptr, 0, n_rows, nodes, capacity,
                                    batch_count, const_cast<float*>(P1), const_cast<float*>(P2),
                                    const_cast<float*>(inv_norm1), const_cast<float*>(inv_norm2),
                                    nullptr, const_cast<float*>(deno), nullptr, workspace,
                                    workspace_bytes);
  t.dE1 = dE1;
  t.ldE1 = ldE1;
  t.dE2 = dE2;
  t.ldE2 = ldE2;
  return hgd::infonce_backward(&t, 1, d, temp, grad_loss, hgd::as_stream(stream),
                               "hgd_infonce_backward_n");
}

extern "C" hgd_status hgd_infonce_forward_group(const hgd_infonce_term* terms, int32_t count,
                                                int32_t d, float temp, void* stream) {
  hgd::clear_error();
  return hgd::infonce_forward(terms, count, d, temp, hgd::as_stream(stream),
                              "hgd_infonce_forward_group");
}

extern "C" hgd_status hgd_infonce_backward_group(const hgd_infonce_term* terms, int32_t count,
                                                 int32_t d, float temp, const float* grad_loss,
                                                 void* stream) {
  hgd::clear_error();
  return hgd::infonce_backward(terms, count, d, temp, grad_loss, hgd::as_stream(stream),
                               "hgd_infonce_backward_group");
}
