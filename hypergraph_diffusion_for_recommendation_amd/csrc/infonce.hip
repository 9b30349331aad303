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
//   * backward: G_bj = g·(exp(s_bj/τ)/deno_b − δ_bj)/(B·τ) is recomputed tile by tile, and
//     dP1 = G·P2, dP2 = Gᵀ·P1 run on the MFMA with the logit tile's accumulator registers used
//     directly as the next MFMA's A operand (rows of the tile on the lane, its columns in the
//     4 registers = the k index, in a permuted order the B operand follows); the split-j partials
//     are summed in order and the F.normalize backward (dx = (dp − p<p,dp>)/‖x‖) is fused into
//     that final pass. The scatter into the [N, d] table gradients is left to the caller.
#include "device_util.h"
#include "hgd_internal.h"

namespace hgd {
namespace {

constexpr float kShift = 1e-8f;   // embeds + 1e-8 (loss_torch.py:104-105)
constexpr float kNormEps = 1e-12f;  // F.normalize eps
constexpr float kDenoEps = 1e-8f;   // ... .sum(-1) + 1e-8 (loss_torch.py:109)

// ---- gather + normalise: one group of G = d/4 lanes per batch row ----
template <int G>
__global__ __launch_bounds__(256) void k_nce_gather(const float* __restrict__ E1, int64_t ld1,
                                                    const float* __restrict__ E2, int64_t ld2,
                                                    const int64_t* __restrict__ nodes, int64_t B,
                                                    int64_t n_rows, int32_t d, float inv_temp,
                                                    float* P1,
                                                    float* P2, float* inv1, float* inv2,
                                                    float* pos_logit, const int64_t* Bp) {
  constexpr int GPB = 256 / G;
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  const int64_t b = static_cast<int64_t>(blockIdx.x) * GPB + g;
  if (b >= B) return;
  if (Bp && b >= *Bp) return;  // a capacity row past the device-side count: never read
  // torch indexing semantics: negative ids count from the end (the reference passes
  // torch.unique(emb.long()), HCCF.py:65-66, which yields -1 / 0 / 1); out-of-range ids are
  // rejected by the caller — clamped here only so that no load leaves the table
  int64_t node = nodes[b];
  if (node < 0) node += n_rows;
  node = node < 0 ? 0 : (node >= n_rows ? n_rows - 1 : node);
  const int c0 = 4 * l;
  const bool ok = c0 < d;
  f32x4 x1 = {0.f, 0.f, 0.f, 0.f}, x2 = {0.f, 0.f, 0.f, 0.f};
  if (ok) {
    x1 = *reinterpret_cast<const f32x4*>(E1 + node * ld1 + c0) + kShift;
    x2 = *reinterpret_cast<const f32x4*>(E2 + node * ld2 + c0) + kShift;
  }
  const float n1 = sqrtf(group_sum<G>(x1.x * x1.x + x1.y * x1.y + x1.z * x1.z + x1.w * x1.w));
  const float n2 = sqrtf(group_sum<G>(x2.x * x2.x + x2.y * x2.y + x2.z * x2.z + x2.w * x2.w));
  const float r1 = 1.f / fmaxf(n1, kNormEps);
  const float r2 = 1.f / fmaxf(n2, kNormEps);
  const f32x4 p1 = x1 * r1, p2 = x2 * r2;
  const float dot = group_sum<G>(p1.x * p2.x + p1.y * p2.y + p1.z * p2.z + p1.w * p2.w);
  if (ok) {
    *reinterpret_cast<f32x4*>(P1 + b * d + c0) = p1;
    *reinterpret_cast<f32x4*>(P2 + b * d + c0) = p2;
  }
  if (l == 0) {
    inv1[b] = r1;
    inv2[b] = r2;
    pos_logit[b] = dot * inv_temp;
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

// ---- forward exp-sums: partial[s][b] = Σ_{j in slice s} exp(<p1_b, p2_j>/τ) ----
// A wave owns 16 rows of p1; the slice's p2 rows stream in 64-row super-tiles (4 MFMA tiles)
// through a copy-free ping-pong, so a super-tile's loads are in flight behind the previous
// one's MFMAs and exps.
template <int DQ>  // d = 4·DQ
__global__ __launch_bounds__(256) void k_nce_rowsum(const float* __restrict__ P1,
                                                    const float* __restrict__ P2, int64_t B,
                                                    float inv_temp, int64_t j_per_slice,
                                                    float* partial, const int64_t* Bp) {
  constexpr int Q4 = DQ / 4;
  constexpr int SUB = 4;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t b0 = static_cast<int64_t>(blockIdx.x) * 64 + 16 * wave;
  const int64_t Be = Bp ? *Bp : B;  // live rows (B is the capacity: strides, clamps)
  if (b0 >= Be) return;
  const int d = 4 * DQ;
  f32x4 a[Q4];
  load_frag4<DQ>(P1, Be, d, b0, lane, a);  // rows clamped to the live ones (the rest unwritten)
  const int64_t j_begin = static_cast<int64_t>(blockIdx.y) * j_per_slice;
  const int64_t j_end = min(Be, j_begin + j_per_slice);
  float psum[4] = {0.f, 0.f, 0.f, 0.f};
  auto load = [&](int64_t j0, f32x4 (&f)[SUB][Q4]) {
#pragma unroll
    for (int t = 0; t < SUB; ++t) load_frag4<DQ>(P2, Be, d, j0 + 16 * t, lane, f[t]);
  };
  auto compute = [&](int64_t j0, const f32x4 (&f)[SUB][Q4]) {
#pragma unroll
    for (int t = 0; t < SUB; ++t) {
      f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < Q4; ++q)
#pragma unroll
        for (int c = 0; c < 4; ++c) s = mfma4(a[q][c], f[t][q][c], s);
      // s[r] = <p1_{b0 + 4(l>>4) + r}, p2_{j0 + 16t + (l&15)}>
      const bool jok = j0 + 16 * t + (lane & 15) < j_end;
#pragma unroll
      for (int r = 0; r < 4; ++r) psum[r] += jok ? expf(s[r] * inv_temp) : 0.f;
    }
  };
  f32x4 f0[SUB][Q4], f1[SUB][Q4];
  int64_t j0 = j_begin;
  load(j0, f0);
  while (j0 < j_end) {
    load(j0 + 16 * SUB, f1);
    __builtin_amdgcn_sched_barrier(0);
    compute(j0, f0);
    __builtin_amdgcn_sched_barrier(0);
    j0 += 16 * SUB;
    if (j0 >= j_end) break;
    load(j0 + 16 * SUB, f0);
    __builtin_amdgcn_sched_barrier(0);
    compute(j0, f1);
    __builtin_amdgcn_sched_barrier(0);
    j0 += 16 * SUB;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) psum[r] = group_sum<16>(psum[r]);
  if ((lane & 15) == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t b = b0 + 4 * (lane >> 4) + r;
      if (b < Be) partial[static_cast<int64_t>(blockIdx.y) * B + b] = psum[r];
    }
  }
}

// ---- finish: deno_b, loss = -(1/B) Σ_b log(exp(pos_b) / deno_b), fixed-order reductions ----
__global__ __launch_bounds__(1024) void k_nce_finish(const float* __restrict__ partial,
                                                     int64_t S, int64_t B,
                                                     const float* __restrict__ pos_logit,
                                                     float* deno, float* loss,
                                                     const int64_t* Bp) {
  __shared__ float red[1024];
  const int64_t Be = Bp ? *Bp : B;
  float acc = 0.f;
  for (int64_t b = threadIdx.x; b < Be; b += 1024) {
    float den = 0.f;
    for (int64_t s = 0; s < S; ++s) den += partial[s * B + b];
    den += kDenoEps;
    deno[b] = den;
    acc += logf(expf(pos_logit[b]) / den);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 512; w >= 1; w >>= 1) {
    if (static_cast<int>(threadIdx.x) < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = -red[0] / static_cast<float>(Be);
}

// ---- backward partials ----
// ROWS = true : part[s][b][:] = Σ_{j in slice s} G_bj p2_j       (dP1)
// ROWS = false: part[s][j][:] = Σ_{b in slice s} G_bj p1_b       (dP2)
// with G_bj = coef·(exp(s_bj/τ)/deno_b − δ_bj), coef = g/(B·τ).
template <int DQ, bool ROWS>
__global__ __launch_bounds__(256) void k_nce_bwd(const float* __restrict__ P1,
                                                 const float* __restrict__ P2, int64_t B,
                                                 float inv_temp, const float* __restrict__ deno,
                                                 const float* __restrict__ grad, float temp,
                                                 int64_t k_per_slice, float* part,
                                                 const int64_t* Bp) {
  constexpr int Q4 = DQ / 4;
  constexpr int SUB = 2;  // 16-row tiles of the streamed matrix per ping-pong stage
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int d = 4 * DQ;
  const int64_t Be = Bp ? *Bp : B;  // live rows (B is the capacity: strides, clamps)
  // upstream dL/dloss and the 1/(B·τ) of the mean: device values, no host sync
  const float coef = grad[0] / (static_cast<float>(Be) * temp);
  // "own" rows: b (ROWS) or j (!ROWS); "other" rows are streamed in 16-row tiles
  const float* own_m = ROWS ? P1 : P2;
  const float* oth_m = ROWS ? P2 : P1;
  const int64_t o0 = static_cast<int64_t>(blockIdx.x) * 64 + 16 * wave;
  if (o0 >= Be) return;
  f32x4 own[Q4];
  load_frag4<DQ>(own_m, Be, d, o0, lane, own);  // rows clamped to the live ones
  const int64_t o_lane = o0 + (lane & 15);  // own row of this lane in the logit tile below
  float deno_own = 1.f;
  if (ROWS) deno_own = deno[o_lane < Be ? o_lane : Be - 1];
  const int64_t k_begin = static_cast<int64_t>(blockIdx.y) * k_per_slice;
  const int64_t k_end = min(Be, k_begin + k_per_slice);
  f32x4 acc[DQ / 4];
#pragma unroll
  for (int t = 0; t < DQ / 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // per 16-row tile: the other rows as logit fragments (row on the lane) and as the B operand of
  // the accumulation (feature on the lane): bv[r][t] = oth[k0 + 4(l>>4) + r][16t + (l&15)]
  struct Tile {
    f32x4 of[Q4];
    float bv[4][DQ / 4];
  };
  auto load = [&](int64_t k0, Tile (&T)[SUB]) {
#pragma unroll
    for (int u = 0; u < SUB; ++u) {
      const int64_t kt = k0 + 16 * u;
      load_frag4<DQ>(oth_m, Be, d, kt, lane, T[u].of);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int64_t k = kt + 4 * (lane >> 4) + r;
        k = k < Be ? k : Be - 1;
#pragma unroll
        for (int t = 0; t < DQ / 4; ++t) T[u].bv[r][t] = oth_m[k * d + 16 * t + (lane & 15)];
      }
    }
  };
  auto compute = [&](int64_t k0, const Tile (&T)[SUB]) {
#pragma unroll
    for (int u = 0; u < SUB; ++u) {
      const int64_t kt = k0 + 16 * u;
      // logit tile with the OTHER index on the output rows:
      // s[r] = <oth_{kt + 4(l>>4) + r}, own_{o0 + (l&15)}>
      f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < Q4; ++q)
#pragma unroll
        for (int c = 0; c < 4; ++c) s = mfma4(T[u].of[q][c], own[q][c], s);
      float gk[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t k = kt + 4 * (lane >> 4) + r;  // other index of register r
        const bool kok = k < k_end;
        const int64_t kc = k < Be ? k : Be - 1;
        const float e = expf(s[r] * inv_temp);
        const float den = ROWS ? deno_own : deno[kc];
        const float delta = (k == o_lane) ? 1.f : 0.f;
        gk[r] = (kok && o_lane < Be) ? coef * (e / den - delta) : 0.f;
      }
      // acc[own row][n] += Σ_k G[own][k]·oth_k[n]: A operand = gk (own row on the lane, k-step
      // r covers other rows {4(l>>4) + r}), B operand = those rows' features (bv).
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int t = 0; t < DQ / 4; ++t) acc[t] = mfma4(gk[r], T[u].bv[r][t], acc[t]);
    }
  };
  Tile t0[SUB], t1[SUB];
  int64_t k0 = k_begin;
  load(k0, t0);
  while (k0 < k_end) {
    load(k0 + 16 * SUB, t1);
    __builtin_amdgcn_sched_barrier(0);
    compute(k0, t0);
    __builtin_amdgcn_sched_barrier(0);
    k0 += 16 * SUB;
    if (k0 >= k_end) break;
    load(k0 + 16 * SUB, t0);
    __builtin_amdgcn_sched_barrier(0);
    compute(k0, t1);
    __builtin_amdgcn_sched_barrier(0);
    k0 += 16 * SUB;
  }
  // acc[t] reg r: own row o0 + 4(l>>4) + r, feature 16t + (l&15)
#pragma unroll
  for (int t = 0; t < DQ / 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t o = o0 + 4 * (lane >> 4) + r;
      if (o < Be) part[(static_cast<int64_t>(blockIdx.y) * B + o) * d + 16 * t + (lane & 15)] =
          acc[t][r];
    }
}

// ---- sum the split partials in order and apply the F.normalize backward per row ----
template <int G>
__global__ __launch_bounds__(256) void k_nce_norm_bwd(const float* __restrict__ part, int64_t S,
                                                      int64_t B, int32_t d,
                                                      const float* __restrict__ P,
                                                      const float* __restrict__ inv, float* dX,
                                                      const int64_t* Bp,
                                                      const int64_t* __restrict__ nodes,
                                                      int64_t n_rows, float* dE, int64_t ldE) {
  constexpr int GPB = 256 / G;
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  const int64_t b = static_cast<int64_t>(blockIdx.x) * GPB + g;
  if (b >= B) return;
  const int c0 = 4 * l;
  const bool ok = c0 < d;
  if (Bp && b >= *Bp) {  // capacity row: a zero gradient row, or nothing to scatter
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
    int64_t node = nodes[b];
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

hgd_status infonce_forward(const float* E1, int64_t ld1, const float* E2, int64_t ld2,
                           int64_t n_rows, const int64_t* nodes, int64_t batch,
                           const int64_t* batch_count, int32_t d, float temp, float* P1,
                           float* P2, float* inv_norm1, float* inv_norm2, float* pos_logit,
                           float* deno, float* loss, void* workspace, size_t workspace_bytes,
                           void* stream) {
  HGD_REQUIRE(batch > 0 && n_rows > 0, "hgd_infonce_forward: empty batch or table");
  HGD_REQUIRE(d % 16 == 0 && d >= 16 && d <= 256,
              "hgd_infonce_forward: d = %d must be a multiple of 16 in [16, 256]", d);
  HGD_REQUIRE(temp > 0.f, "hgd_infonce_forward: temperature must be > 0");
  HGD_REQUIRE(ld1 >= d && ld2 >= d && ld1 % 4 == 0 && ld2 % 4 == 0,
              "hgd_infonce_forward: leading dimensions must be >= d and multiples of 4");
  HGD_REQUIRE(E1 && E2 && nodes && P1 && P2 && inv_norm1 && inv_norm2 && pos_logit && deno && loss,
              "hgd_infonce_forward: null pointer");
  HGD_REQUIRE(reinterpret_cast<uintptr_t>(E1) % 16 == 0 && reinterpret_cast<uintptr_t>(E2) % 16 == 0,
              "hgd_infonce_forward: tables must be 16-byte aligned");
  const size_t need = hgd_infonce_workspace_size(batch, d);
  if (workspace_bytes < need || !workspace)
    return fail(HGD_ERR_WORKSPACE, "hgd_infonce_forward: workspace %zu < required %zu",
                workspace_bytes, need);
  hipStream_t st = as_stream(stream);
  const float inv_temp = 1.f / temp;
  const int G = group_for(d);
  const int64_t gpb = 256 / G;
  const dim3 gg(static_cast<unsigned>((batch + gpb - 1) / gpb));
  switch (G) {
    case 4: hipLaunchKernelGGL((k_nce_gather<4>), gg, dim3(256), 0, st, E1, ld1, E2, ld2, nodes, batch, n_rows, d, inv_temp, P1, P2, inv_norm1, inv_norm2, pos_logit, batch_count); break;
    case 8: hipLaunchKernelGGL((k_nce_gather<8>), gg, dim3(256), 0, st, E1, ld1, E2, ld2, nodes, batch, n_rows, d, inv_temp, P1, P2, inv_norm1, inv_norm2, pos_logit, batch_count); break;
    case 16: hipLaunchKernelGGL((k_nce_gather<16>), gg, dim3(256), 0, st, E1, ld1, E2, ld2, nodes, batch, n_rows, d, inv_temp, P1, P2, inv_norm1, inv_norm2, pos_logit, batch_count); break;
    case 32: hipLaunchKernelGGL((k_nce_gather<32>), gg, dim3(256), 0, st, E1, ld1, E2, ld2, nodes, batch, n_rows, d, inv_temp, P1, P2, inv_norm1, inv_norm2, pos_logit, batch_count); break;
    default: hipLaunchKernelGGL((k_nce_gather<64>), gg, dim3(256), 0, st, E1, ld1, E2, ld2, nodes, batch, n_rows, d, inv_temp, P1, P2, inv_norm1, inv_norm2, pos_logit, batch_count); break;
  }
  hgd_status s = check_launch("hgd_infonce_forward gather");
  if (s != HGD_OK) return s;
  const int64_t S = slices_for(batch);
  const int64_t jps = per_slice(batch, S);
  const int64_t S_used = (batch + jps - 1) / jps;
  float* partial = static_cast<float*>(workspace);
  const dim3 gr(static_cast<unsigned>((batch + 63) / 64), static_cast<unsigned>(S_used));
  switch (d / 4) {
#define HGD_CASE(DQ)                                                                              \
    case DQ:                                                                                      \
      hipLaunchKernelGGL((k_nce_rowsum<DQ>), gr, dim3(256), 0, st, P1, P2, batch, inv_temp, jps, \
                         partial, batch_count);                                                   \
      break;
    HGD_CASE(4) HGD_CASE(8) HGD_CASE(12) HGD_CASE(16) HGD_CASE(20) HGD_CASE(24) HGD_CASE(28)
    HGD_CASE(32) HGD_CASE(36) HGD_CASE(40) HGD_CASE(44) HGD_CASE(48) HGD_CASE(52) HGD_CASE(56)
    HGD_CASE(60) HGD_CASE(64)
#undef HGD_CASE
    default: return fail(HGD_ERR_UNSUPPORTED, "hgd_infonce_forward: d = %d", d);
  }
  s = check_launch("hgd_infonce_forward rowsum");
  if (s != HGD_OK) return s;
  hipLaunchKernelGGL(k_nce_finish, dim3(1), dim3(1024), 0, st, partial, S_used, batch, pos_logit,
                     deno, loss, batch_count);
  return check_launch("hgd_infonce_forward finish");
}


hgd_status infonce_backward(const float* P1, const float* P2, const float* inv_norm1,
                            const float* inv_norm2, const float* deno, int64_t batch,
                            const int64_t* batch_count, int32_t d, float temp,
                            const float* grad_loss, float* dX1, float* dX2,
                            const int64_t* nodes, int64_t n_rows, float* dE1, int64_t ldE1,
                            float* dE2, int64_t ldE2, void* workspace,
                            size_t workspace_bytes, void* stream) {
  HGD_REQUIRE(batch > 0, "hgd_infonce_backward: empty batch");
  HGD_REQUIRE(d % 16 == 0 && d >= 16 && d <= 256,
              "hgd_infonce_backward: d = %d must be a multiple of 16 in [16, 256]", d);
  HGD_REQUIRE(temp > 0.f, "hgd_infonce_backward: temperature must be > 0");
  HGD_REQUIRE(P1 && P2 && inv_norm1 && inv_norm2 && deno && grad_loss,
              "hgd_infonce_backward: null pointer");
  const bool side1 = dX1 || dE1, side2 = dX2 || dE2;  // a side without an output is skipped
  HGD_REQUIRE(side1 || side2, "hgd_infonce_backward: no output");
  HGD_REQUIRE(!(dE1 || dE2) || (nodes && n_rows > 0 && (!dE1 || ldE1 >= d) &&
                                (!dE2 || ldE2 >= d)),
              "hgd_infonce_backward: a table scatter needs nodes, n_rows and ld >= d");
  const size_t need = hgd_infonce_workspace_size(batch, d);
  if (workspace_bytes < need || !workspace)
    return fail(HGD_ERR_WORKSPACE, "hgd_infonce_backward: workspace %zu < required %zu",
                workspace_bytes, need);
  hipStream_t st = as_stream(stream);
  const float inv_temp = 1.f / temp;
  const int64_t S = slices_for(batch);
  const int64_t kps = per_slice(batch, S);
  const int64_t S_used = (batch + kps - 1) / kps;
  char* ws = static_cast<char*>(workspace);
  const size_t off = align_up(static_cast<size_t>(S) * batch * 4);
  float* part1 = reinterpret_cast<float*>(ws + off);
  float* part2 = reinterpret_cast<float*>(ws + off + align_up(static_cast<size_t>(S) * batch * d * 4));
  const dim3 gr(static_cast<unsigned>((batch + 63) / 64), static_cast<unsigned>(S_used));
  switch (d / 4) {
#define HGD_CASE(DQ)                                                                              \
    case DQ:                                                                                      \
      if (side1)                                                                                  \
        hipLaunchKernelGGL((k_nce_bwd<DQ, true>), gr, dim3(256), 0, st, P1, P2, batch, inv_temp, \
                           deno, grad_loss, temp, kps, part1, batch_count);                        \
      if (side2)                                                                                  \
        hipLaunchKernelGGL((k_nce_bwd<DQ, false>), gr, dim3(256), 0, st, P1, P2, batch,          \
                           inv_temp, deno, grad_loss, temp, kps, part2, batch_count);              \
      break;
    HGD_CASE(4) HGD_CASE(8) HGD_CASE(12) HGD_CASE(16) HGD_CASE(20) HGD_CASE(24) HGD_CASE(28)
    HGD_CASE(32) HGD_CASE(36) HGD_CASE(40) HGD_CASE(44) HGD_CASE(48) HGD_CASE(52) HGD_CASE(56)
    HGD_CASE(60) HGD_CASE(64)
#undef HGD_CASE
    default: return fail(HGD_ERR_UNSUPPORTED, "hgd_infonce_backward: d = %d", d);
  }
  hgd_status s = check_launch("hgd_infonce_backward partials");
  if (s != HGD_OK) return s;
  const int G = group_for(d);
  const int64_t gpb = 256 / G;
  const dim3 gn(static_cast<unsigned>((batch + gpb - 1) / gpb));
  switch (G) {
#define HGD_CASE(GG)                                                                         \
    case GG:                                                                                 \
      if (side1)                                                                             \
        hipLaunchKernelGGL((k_nce_norm_bwd<GG>), gn, dim3(256), 0, st, part1, S_used, batch, \
                           d, P1, inv_norm1, dX1, batch_count, nodes, n_rows, dE1, ldE1);    \
      if (side2)                                                                             \
        hipLaunchKernelGGL((k_nce_norm_bwd<GG>), gn, dim3(256), 0, st, part2, S_used, batch, \
                           d, P2, inv_norm2, dX2, batch_count, nodes, n_rows, dE2, ldE2);    \
      break;
    HGD_CASE(4) HGD_CASE(8) HGD_CASE(16) HGD_CASE(32) HGD_CASE(64)
#undef HGD_CASE
    default: return fail(HGD_ERR_UNSUPPORTED, "hgd_infonce_backward: group %d", G);
  }
  return check_launch("hgd_infonce_backward norm");
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
  return hgd::infonce_forward(E1, ld1, E2, ld2, n_rows, nodes, batch, nullptr, d, temp, P1, P2,
                              inv_norm1, inv_norm2, pos_logit, deno, loss, workspace,
                              workspace_bytes, stream);
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
  return hgd::infonce_forward(E1, ld1, E2, ld2, n_rows, nodes, capacity, batch_count, d, temp,
                              P1, P2, inv_norm1, inv_norm2, pos_logit, deno, loss, workspace,
                              workspace_bytes, stream);
}

extern "C" hgd_status hgd_infonce_backward(const float* P1, const float* P2,
                                           const float* inv_norm1, const float* inv_norm2,
                                           const float* deno, int64_t batch, int32_t d,
                                           float temp, const float* grad_loss, float* dX1,
                                           float* dX2, void* workspace, size_t workspace_bytes,
                                           void* stream) {
  hgd::clear_error();
  HGD_REQUIRE(dX1 && dX2, "hgd_infonce_backward: null dX1/dX2");
  return hgd::infonce_backward(P1, P2, inv_norm1, inv_norm2, deno, batch, nullptr, d, temp,
                               grad_loss, dX1, dX2, nullptr, 0, nullptr, 0, nullptr, 0,
                               workspace, workspace_bytes, stream);
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
  return hgd::infonce_backward(P1, P2, inv_norm1, inv_norm2, deno, capacity, batch_count, d,
                               temp, grad_loss, nullptr, nullptr, nodes, n_rows, dE1, ldE1, dE2,
                               ldE2, workspace, workspace_bytes, stream);
}
