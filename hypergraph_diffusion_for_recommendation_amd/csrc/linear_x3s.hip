// The staged split-bf16 row GEMM (k_row_gemm_x3s), built once per K = 32·HGD_X3S_KQ (the Makefile
// compiles this file four times): the dense forward / backward-data products of SURVEY.md §8f
// rank 1 (lin_in, EquivSetGNN2.py:91-94; MLP layers, model/layers/MLP.py:109-117). The split-bf16
// arithmetic and its error bound are described in linear.hip.
#include <algorithm>

#include "linear_common.h"

#ifndef HGD_X3S_KQ
#error "linear_x3s.hip is compiled with -DHGD_X3S_KQ=1..4"
#endif

namespace hgd {
namespace lin {
namespace {

// ---------------------------------------------------------------------------------------------
// Staged split-bf16 row GEMM (the default form). k_row_gemm_x3 loads each lane's MFMA fragment
// straight from HBM (16 rows × 64 B per instruction: half lines, the TA's worst case), splits it
// in every wave that needs it and re-reads all of W's planes from LDS for each 16-row tile: at
// 144 k × 128 → 128 it ran 43 µs, MFMA-issue 25 % busy. Here, per workgroup of WAVES waves:
//
//  * the activation rows stream through a register ring D stages deep, in whole 128-B lines
//    (consecutive lanes, consecutive 16-B pieces of a row: 1 KB per wave instruction), each
//    float4 loaded by exactly one thread;
//  * that thread applies the input dropout / ReLU mask / binarization, splits its four values
//    into the three bf16 terms and writes them to the stage's planes in LDS in MFMA-fragment
//    order (slot g·16 + (j ^ (4g + q)) of the row tile's q-block: conflict-free 8-byte writes
//    for the 32 lanes of a row, conflict-free 16-byte fragment reads); the row sums for row_inv
//    are a shuffle reduction over the lanes holding the row;
//  * wave (rt, cg) computes row tile rt × column group cg (NTW 16-column tiles) of the stage
//    with its W fragments held in REGISTERS (split once per workgroup), so the only LDS reads
//    are three activation fragments per k step, shared by its NTW·6 MFMAs;
//  * one barrier per stage (two plane buffers), the residual / accumulate rows of the stage
//    requested before its ring refill so that waiting for them never waits for the refill.
//
// R = 16·RT rows per stage; K = 32·KQ; THREADS = 64·CG·RT. EPI: 0 plain store, 1 the second
// store Y2 = Y + res, 2 accumulate (Y += product) — template arguments, so that no load of the
// stage sits in a runtime branch (hipcc then waits vmcnt(0) at the join, draining the ring).
template <int KQ, int NTW, int CG, int RT, bool MASK>
struct X3S {
  static constexpr int K = 32 * KQ;
  static constexpr int R = 16 * RT;
  static constexpr int WAVES = CG * RT;
  static constexpr int THREADS = 64 * WAVES;
  static constexpr int F4 = R * K / 4;                       // float4 pieces of a stage
  static constexpr int F = (F4 + THREADS - 1) / THREADS;     // per thread
  // ring depth: 8 float4 pieces (128 B) per thread in flight — 64 KB per 8-wave workgroup
  static constexpr int D = F >= 8 ? 1 : 8 / F;
  static constexpr int LPR = K / 4;                          // lanes holding one row
  static constexpr size_t PLANE_BYTES = static_cast<size_t>(RT) * KQ * 1024;  // one plane, one stage
  static constexpr size_t PLANES_LDS = 2 * 3 * PLANE_BYTES + 2 * R * 4;
  static constexpr size_t W_LDS = static_cast<size_t>(K) * (16 * CG * NTW + 4) * 4;  // staging
  static constexpr size_t LDS = PLANES_LDS > W_LDS ? PLANES_LDS : W_LDS;
};

template <int KQ, int NTW, int CG, int RT, bool MASK, int EPI>
__global__ __launch_bounds__(64 * CG * RT) void k_row_gemm_x3s(RowGemmGroup grp) {
  using C = X3S<KQ, NTW, CG, RT, MASK>;
  extern __shared__ __attribute__((aligned(16))) char x3s_smem[];
  char* planes = x3s_smem;                                            // [2][3][RT][KQ][1 KB]
  float* s_inv = reinterpret_cast<float*>(x3s_smem + 2 * 3 * C::PLANE_BYTES);  // [2][R]
  int bxg, ys;
  row_block_of(grp, bxg, ys);
  const bool second = grp.count > 1 && bxg >= grp.nb0;
  const RowGemm p = second ? grp.p[1] : grp.p[0];
  const int bx = bxg - (second ? grp.nb0 : 0);
  const int nbx = grp.count > 1 ? (second ? grp.nbt - grp.nb0 : grp.nb0) : grp.nbt;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int i16 = lane & 15;
  const int g = lane >> 4;
  const int rt = wave % RT, cg = wave / RT;
  constexpr int NTS = CG * NTW;  // 16-column tiles per slice
  const int n0 = ys * 16 * NTS;
  const int nt = min(NTS, (p.N - n0) / 16);  // live tiles of this slice
  const int64_t stages = (p.rows + C::R - 1) / C::R;

  // ---- the ring: stage i of this workgroup is row block bx + i·nbx. Its first D stages are
  // requested before W is staged, so the two latencies overlap.
  f32x4 raw[C::D][C::F], rawm[C::D][C::F];
  auto ring_load = [&](int64_t i, f32x4 (&a)[C::F], f32x4 (&m)[C::F]) {
    int64_t sb = static_cast<int64_t>(bx) + i * nbx;
    sb = sb < stages ? sb : stages - 1;  // past the end: a valid block, never consumed
#pragma unroll
    for (int u = 0; u < C::F; ++u) {
      int f = tid + C::THREADS * u;
      f = f < C::F4 ? f : C::F4 - 1;
      int64_t row = sb * C::R + f / C::LPR;
      row = row < p.rows ? row : p.rows - 1;
      const int c = f % C::LPR;
      a[u] = ld4(p.A + row * p.lda + 4 * c);
      if constexpr (MASK) m[u] = ld4(p.mask + row * p.ldm + 4 * c);
    }
  };
#pragma unroll
  for (int d = 0; d < C::D; ++d) ring_load(d, raw[d], rawm[d]);

  // ---- W's slice → LDS (coalesced along whichever of k / n is contiguous in memory, scaled
  // there), then each wave's fragments (tile t = cg·NTW + tw, k step q, planes 0..2) → registers.
  // All loads of a kind are issued before any is used: a load under a runtime condition inside
  // an element loop made hipcc wait vmcnt(0) after each one.
  bf16x8 wf[NTW][KQ][3];
  f32x4 bias4[NTW];
  {
    constexpr int NSL = 16 * NTS;                 // slice columns
    constexpr int LDW = NSL + 4;                  // padded LDS row of k
    constexpr int EW = (C::K * NSL + C::THREADS - 1) / C::THREADS;
    static_assert(C::K * LDW * 4 <= C::LDS, "W staging must fit the kernel's LDS");
    float* sWt = reinterpret_cast<float*>(x3s_smem);  // [K][LDW], before the planes are used
    const bool kfast = p.bsk == 1;
    // chunks of 8 elements per thread: 8 loads in flight without holding all EW in registers
    // (the staging phase set the kernel's register peak, on top of the ring)
    constexpr int CH = EW < 8 ? EW : 8;
#pragma unroll 1
    for (int r0 = 0; r0 < EW; r0 += CH) {
      float wv[CH];
      int ek[CH], en[CH];
#pragma unroll
      for (int r = 0; r < CH; ++r) {
        int e = tid + C::THREADS * (r0 + r);
        e = e < C::K * NSL ? e : C::K * NSL - 1;
        ek[r] = kfast ? e % C::K : e / NSL;
        en[r] = kfast ? e / C::K : e % NSL;
        const int n = n0 + en[r] < p.N ? n0 + en[r] : p.N - 1;
        wv[r] = p.B[static_cast<int64_t>(ek[r]) * p.bsk + static_cast<int64_t>(n) * p.bsn];
      }
      if (p.b_row_count) {
        float cnt[CH];
#pragma unroll
        for (int r = 0; r < CH; ++r) cnt[r] = p.b_row_count[ek[r]];
#pragma unroll
        for (int r = 0; r < CH; ++r) wv[r] *= 1.f / fmaxf(cnt[r], 1.f);
      }
#pragma unroll
      for (int r = 0; r < CH; ++r) {
        float w = wv[r];
        if (p.b_scale != 0.f) w *= p.b_scale;
        if (n0 + en[r] >= p.N) w = 0.f;
        if (r0 + r < EW && tid + C::THREADS * (r0 + r) < C::K * NSL) sWt[ek[r] * LDW + en[r]] = w;
      }
    }
    __syncthreads();
#pragma unroll
    for (int tw = 0; tw < NTW; ++tw) {
      const int col = 16 * (cg * NTW + tw) + i16;
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          v[j] = sWt[(32 * q + (j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4))) * LDW + col];
        split3(v, wf[tw][q][0], wf[tw][q][1], wf[tw][q][2]);
      }
    }
    float bv[NTW][4];
#pragma unroll
    for (int tw = 0; tw < NTW; ++tw) {
      const int t = cg * NTW + tw;
      const int c0 = n0 + 16 * (t < nt ? t : 0) + 4 * g;
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) bv[tw][cc] = p.bias ? p.bias[c0 + cc] : 0.f;
      bias4[tw] = t < nt ? f32x4{bv[tw][0], bv[tw][1], bv[tw][2], bv[tw][3]}
                         : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();  // the staging region becomes plane buffers
  }

  const uint64_t drop_seed = p.drop_seed ? *p.drop_seed : 0ull;
  const uint32_t drop_thr = dropout_threshold(p.drop_keep);
  const uint64_t a_seed = p.a_drop_seed ? *p.a_drop_seed : 0ull;
  const uint32_t a_thr = dropout_threshold(p.a_drop_keep);

  auto stage = [&](int64_t i, int buf, f32x4 (&a)[C::F], f32x4 (&m)[C::F]) {
    const int64_t sb = static_cast<int64_t>(bx) + i * nbx;
    const int64_t r0 = sb * C::R;
    // (1) this wave's output rows: residual / accumulate pieces, requested before the refill
    const int64_t orow = r0 + 16 * rt + i16;
    const bool olive = orow < p.rows;
    const int64_t orc = olive ? orow : p.rows - 1;
    f32x4 ev[NTW];  // EPI 1: residual pieces, EPI 2: the Y pieces the product is added to
    if constexpr (EPI != kEpiPlain) {
#pragma unroll
      for (int tw = 0; tw < NTW; ++tw) {
        const int t = cg * NTW + tw;
        const int col = n0 + 16 * (t < nt ? t : 0) + 4 * g;
        ev[tw] = EPI == kEpiRes ? ld4(p.res + orc * p.ldres + col) : ld4(p.Y + orc * p.ldy + col);
      }
    }
    // (2) split this thread's pieces into the stage's planes (+ row sums for row_inv)
    char* pb = planes + static_cast<size_t>(buf) * 3 * C::PLANE_BYTES;
#pragma unroll
    for (int u = 0; u < C::F; ++u) {
      const int f = tid + C::THREADS * u;
      if (C::F4 % C::THREADS != 0 && f >= C::F4) continue;
      const int rl = f / C::LPR, c = f % C::LPR;
      f32x4 x = a[u];
      if (p.a_drop_seed) {
        const uint32_t e = static_cast<uint32_t>(r0 + rl) * static_cast<uint32_t>(C::K) + 4 * c;
        x = dropout_apply4(x, a_seed, e >> 2, a_thr, p.a_drop_scale);
      }
      if constexpr (MASK) {
        x = relu_mask(x, m[u]);
      } else if (p.binarize_a) {
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) x[cc] = x[cc] > 0.f ? 1.f : 0.f;
      }
      if (!MASK && p.row_inv) {
        float rs = (x.x + x.y) + (x.z + x.w);
#pragma unroll
        for (int o = 1; o < C::LPR; o <<= 1) rs += __shfl_xor(rs, o);
        if (c == 0) s_inv[buf * C::R + rl] = 1.f / fmaxf(rs, 1.f);
      }
      bf16x4 h, md, lo;
      split3x4(x, h, md, lo);
      const int q = c >> 3, e = c & 7, gg = e & 3, half = e >> 2, j = rl & 15;
      const size_t off = (static_cast<size_t>(rl >> 4) * KQ + q) * 1024 +
                         static_cast<size_t>(gg * 16 + (j ^ (4 * gg + q))) * 16 + half * 8;
      *reinterpret_cast<bf16x4*>(pb + off) = h;
      *reinterpret_cast<bf16x4*>(pb + C::PLANE_BYTES + off) = md;
      *reinterpret_cast<bf16x4*>(pb + 2 * C::PLANE_BYTES + off) = lo;
    }
    // (3) refill this ring slot with stage i + D
    ring_load(i + C::D, a, m);
    __syncthreads();
    // the row scale before the MFMAs: the epilogue's first read of the accumulators then sits in
    // the same basic block as the last MFMA. With a branch in between, hipcc (ROCm 7.2) read the
    // accumulator registers without the MFMA→VALU wait states (stale results at NTW = 1, where
    // no second accumulation chain separates them)
    float inv = 1.f;
    if (!MASK && p.row_inv) {
      inv = s_inv[buf * C::R + 16 * rt + i16];
      if (g == 0 && cg == 0 && n0 == 0 && olive) p.row_inv[orow] = inv;
    }
    // (4) MFMAs: this wave's row tile × column group, W in registers
    f32x4 acc[NTW];
#pragma unroll
    for (int tw = 0; tw < NTW; ++tw) acc[tw] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* fb = pb + static_cast<size_t>(rt) * KQ * 1024;
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      const size_t so = static_cast<size_t>(q) * 1024 +
                        static_cast<size_t>(g * 16 + (i16 ^ (4 * g + q))) * 16;
      const bf16x8 xh = *reinterpret_cast<const bf16x8*>(fb + so);
      const bf16x8 xm = *reinterpret_cast<const bf16x8*>(fb + C::PLANE_BYTES + so);
      const bf16x8 xl = *reinterpret_cast<const bf16x8*>(fb + 2 * C::PLANE_BYTES + so);
#pragma unroll
      for (int tw = 0; tw < NTW; ++tw)
        acc[tw] = mfma_x3(wf[tw][q][0], wf[tw][q][1], wf[tw][q][2], xh, xm, xl, acc[tw], false);
    }
    // (5) epilogue: lane (i16, g) holds row orow, columns n0 + 16t + 4g + 0..3; the scale and
    // bias unconditionally (inv = 1 without row_inv: bitwise the unscaled sum) and at once
    mfma_drain();
    f32x4 outv[NTW];
#pragma unroll
    for (int tw = 0; tw < NTW; ++tw) outv[tw] = acc[tw] * inv + bias4[tw];
#pragma unroll
    for (int tw = 0; tw < NTW; ++tw) {
      const int t = cg * NTW + tw;
      const int col = n0 + 16 * t + 4 * g;
      f32x4 v = outv[tw];
      if (p.relu) {
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) v[cc] = v[cc] < 0.f ? 0.f : v[cc];
      }
      if (p.drop_seed) {  // the lane's four columns are one keep group (N % 16 == 0)
        const uint32_t e = static_cast<uint32_t>(orow) * static_cast<uint32_t>(p.N) +
                           static_cast<uint32_t>(col);
        v = dropout_apply4(v, drop_seed, e >> 2, drop_thr, p.drop_scale);
      }
      if (!olive || t >= nt) continue;
      if constexpr (EPI == kEpiAcc) v += ev[tw];
      *reinterpret_cast<f32x4*>(p.Y + orow * p.ldy + col) = v;
      if constexpr (EPI == kEpiRes) *reinterpret_cast<f32x4*>(p.Y2 + orow * p.ldy2 + col) = v + ev[tw];
    }
  };
  // stages of this workgroup, the ring slot index i % D made static by unrolling D stages
  const int64_t my_stages = bx < stages ? (stages - bx + nbx - 1) / nbx : 0;
  // Whole groups of D stages run without a condition, the last partial group after the loop: with
  // the per-stage condition inside the loop, the path that skipped stages left the latest ring
  // load last in the queue, and hipcc's merge at the loop header waited vmcnt(0) — the whole ring
  // drained once per group
  int64_t i0 = 0;
  for (; i0 + C::D <= my_stages; i0 += C::D) {
#pragma unroll
    for (int d = 0; d < C::D; ++d) stage(i0 + d, static_cast<int>((i0 + d) & 1), raw[d], rawm[d]);
  }
  if (i0 < my_stages) {
#pragma unroll
    for (int d = 0; d < C::D; ++d) {
      if (i0 + d < my_stages) stage(i0 + d, static_cast<int>((i0 + d) & 1), raw[d], rawm[d]);
    }
  }
}
// One staged split-bf16 launch (k_row_gemm_x3s): persistent workgroups, at most one resident
// round, shared by a group's products in proportion to their rows; column slices XCD-paired.
template <int KQ, int NTW, int CG, bool MASK, int EPI>
hgd_status launch_x3s(RowGemmGroup g, hipStream_t st, const char* fn) {
  constexpr int RT = (8 / CG) < (16 / KQ) ? (8 / CG) : (16 / KQ) >= 4 ? 4 : 2;
  using C = X3S<KQ, NTW, CG, RT, MASK>;
  const void* kern = reinterpret_cast<const void*>(&k_row_gemm_x3s<KQ, NTW, CG, RT, MASK, EPI>);
  static int resident = 0;
  if (resident == 0) {
    if (C::LDS > 65536)
      HGD_HIP(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  static_cast<int>(C::LDS)));
    int nb = 0, dev = 0, cus = 0;
    HGD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, C::THREADS, C::LDS));
    HGD_HIP(hipGetDevice(&dev));
    HGD_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    resident = std::max(1, nb) * std::max(1, cus);
  }
  int64_t want[2] = {0, 0}, total = 0;
  for (int i = 0; i < g.count; ++i) {
    want[i] = (g.p[i].rows + C::R - 1) / C::R;
    total += want[i];
  }
  g.ny = (g.p[0].N + 16 * CG * NTW - 1) / (16 * CG * NTW);
  const int64_t cap = std::max<int64_t>(1, resident / g.ny);
  int64_t bx[2] = {0, 0};
  for (int i = 0; i < g.count; ++i) {
    bx[i] = total > cap ? std::max<int64_t>(1, want[i] * cap / total) : want[i];
    if (g.ny > 1) bx[i] = (bx[i] + 7) / 8 * 8;
  }
  g.nb0 = static_cast<int32_t>(bx[0]);
  g.nbt = static_cast<int32_t>(bx[0] + bx[1]);
  const dim3 grid(static_cast<unsigned>(g.nbt) * static_cast<unsigned>(g.ny));
  hipLaunchKernelGGL((k_row_gemm_x3s<KQ, NTW, CG, RT, MASK, EPI>), grid, dim3(C::THREADS), C::LDS,
                     st, g);
  return check_launch(fn);
}

template <int KQ, int NTW, int CG>
hgd_status launch_x3s_epi(const RowGemmGroup& g, hipStream_t st, const char* fn) {
  // every product of a group has the same mask mode; the epilogue kind must match too
  const RowGemm& p = g.p[0];
  const int epi = p.Y2 ? kEpiRes : (p.accumulate ? kEpiAcc : kEpiPlain);
  for (int i = 1; i < g.count; ++i) {
    const RowGemm& q = g.p[i];
    HGD_REQUIRE((q.Y2 ? kEpiRes : (q.accumulate ? kEpiAcc : kEpiPlain)) == epi,
                "%s: grouped products need the same epilogue (residual / accumulate)", fn);
  }
  if (p.mask) {
    if (epi == kEpiAcc) return launch_x3s<KQ, NTW, CG, true, kEpiAcc>(g, st, fn);
    return launch_x3s<KQ, NTW, CG, true, kEpiPlain>(g, st, fn);
  }
  if (epi == kEpiRes) return launch_x3s<KQ, NTW, CG, false, kEpiRes>(g, st, fn);
  if (epi == kEpiAcc) return launch_x3s<KQ, NTW, CG, false, kEpiAcc>(g, st, fn);
  return launch_x3s<KQ, NTW, CG, false, kEpiPlain>(g, st, fn);
}

template <int KQ>
hgd_status launch_x3s_shape(const RowGemmGroup& g, hipStream_t st, const char* fn) {
  const int nt = (std::min(g.p[0].N, 128) + 15) / 16;
  if (nt <= 1) return launch_x3s_epi<KQ, 1, 1>(g, st, fn);
  if (nt <= 2) return launch_x3s_epi<KQ, 2, 1>(g, st, fn);
  if (nt <= 4) return launch_x3s_epi<KQ, 2, 2>(g, st, fn);
  return launch_x3s_epi<KQ, 2, 4>(g, st, fn);
}

}  // namespace

template <>
hgd_status launch_x3s_k<HGD_X3S_KQ>(const RowGemmGroup& g, hipStream_t st, const char* fn) {
  return launch_x3s_shape<HGD_X3S_KQ>(g, st, fn);
}

}  // namespace lin
}  // namespace hgd
