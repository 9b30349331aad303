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
//    order: row j's k-group g of q-block q in 16-byte slot g·16 + (j ^ (2g + (q & 1))). On gfx950
//    ds_read_b128 serves lanes in 4 groups of 16 ({0–3,12–15,20–27}, {4–11,16–19,28–31}, …;
//    bank = dword mod 64) and ds_write_b64 in 4 groups of 16 consecutive lanes (dword mod 32):
//    with this swizzle both the fragment reads and the 8-byte plane writes are conflict-free
//    (the earlier j ^ (4g + q) left both 2-way: 4.6 M conflict cycles per launch at d = 128);
//    the row sums for row_inv are a shuffle reduction over the lanes holding the row;
//  * wave (rt, cg) computes row tile rt × column group cg (NTW 16-column tiles) of the stage
//    with its W fragments held in REGISTERS (split once per workgroup), so the only LDS reads
//    are three activation fragments per k step, shared by its NTW·6 MFMAs;
//  * one barrier per stage (two plane buffers), the residual / accumulate rows of the stage
//    requested before its ring refill so that waiting for them never waits for the refill.
//
// R = 16·RT rows per stage; K = 32·KQ; THREADS = 64·CG·RT. EPI: 0 plain store, 1 the second
// store Y2 = Y + res, 2 accumulate (Y += product) — template arguments, so that no load of the
// stage sits in a runtime branch (hipcc then waits vmcnt(0) at the join, draining the ring).
template <int KQ, int NTW, int CG, int RT, bool MASK, int PW>
struct X3S {
  static constexpr int K = 32 * KQ;
  static constexpr int R = 16 * RT;
  static constexpr int CWAVES = CG * RT;                     // waves computing tiles
  static constexpr int WAVES = CWAVES + PW;                  // + producer waves (PW > 0)
  static constexpr int THREADS = 64 * WAVES;
  static constexpr int STHREADS = PW > 0 ? 64 * PW : THREADS;  // threads loading and splitting
  static constexpr int F4 = R * K / 4;                       // float4 pieces of a stage
  static constexpr int F = (F4 + STHREADS - 1) / STHREADS;   // per loading thread
  // ring depth: 8 float4 pieces (128 B) per thread in flight — 64 KB per 8-wave workgroup; with
  // one column tile per wave (two workgroups per CU in 128 registers) 6 pieces, 2 with a mask;
  // producer waves (no W registers) 12, 4 with a mask — 48 KB per workgroup
  static constexpr int RING = PW > 0 ? (MASK ? 4 : 12) : NTW == 1 ? (MASK ? 2 : 6) : 8;
  static constexpr int D = F >= RING ? 1 : RING / F;
  static constexpr int LPR = K / 4;                          // lanes holding one row
  static constexpr size_t PLANE_BYTES = static_cast<size_t>(RT) * KQ * 1024;  // one plane, one stage
  static constexpr size_t PLANES_LDS = 2 * 3 * PLANE_BYTES + 2 * R * 4;
  // W staging, [k][n + 4] or [n][k + pad ≡ 8 mod 64] floats (the larger of the two)
  static constexpr size_t W_KN = static_cast<size_t>(K) * (16 * CG * NTW + 4) * 4;
  static constexpr size_t W_NK = static_cast<size_t>(16 * CG * NTW) * (K + ((8 - K) % 64 + 64) % 64) * 4;
  static constexpr size_t W_LDS = W_KN > W_NK ? W_KN : W_NK;
  static constexpr size_t LDS = PLANES_LDS > W_LDS ? PLANES_LDS : W_LDS;
};

// SPL: what the split applies besides the ReLU mask — kSplPlain nothing, kSplDrop the input
// dropout, kSplAny the runtime flags (dropout, binarization, row_inv) in branches
constexpr int kSplPlain = 0, kSplDrop = 1, kSplAny = 2;

// PW > 0: PW producer waves load the row blocks and split them into the planes while the CG·RT
// consumer waves run the MFMAs and epilogues of the previous stage (one barrier per stage); the
// two phases then overlap across waves instead of alternating inside every wave.
template <int KQ, int NTW, int CG, int RT, bool MASK, int EPI, int SPL, int PW>
__global__ __launch_bounds__(64 * (CG * RT + PW))
__attribute__((amdgpu_waves_per_eu(PW > 0 ? 3 : NTW == 1 && CG >= 4 ? 4 : 1)))
void k_row_gemm_x3s(RowGemmGroup grp) {
  using C = X3S<KQ, NTW, CG, RT, MASK, PW>;
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
  const int rt = wave % RT, cg = (wave / RT) % CG;
  const bool producer = PW > 0 && wave >= C::CWAVES;
  const int stid = PW > 0 ? tid - 64 * C::CWAVES : tid;  // index among the loading threads
  constexpr int NTS = CG * NTW;  // 16-column tiles per slice
  const int n0 = ys * 16 * NTS;
  const int nt = min(NTS, (p.N - n0) / 16);  // live tiles of this slice
  const int64_t stages = (p.rows + C::R - 1) / C::R;

  // ---- the ring: stage i of this workgroup is row block bx + i·nbx. Its first D stages are
  // requested before W is staged, so the two latencies overlap.
  // per-lane byte offsets within a stage's row block (the same for every stage)
  uint32_t aoff[C::F], moff[C::F];
#pragma unroll
  for (int u = 0; u < C::F; ++u) {
    const int f = stid + C::STHREADS * u;
    const uint32_t rl = f / C::LPR, c = f % C::LPR;
    aoff[u] = f < C::F4 ? (rl * static_cast<uint32_t>(p.lda) + 4 * c) * 4 : kBufOff;
    moff[u] = f < C::F4 ? (rl * static_cast<uint32_t>(p.ldm) + 4 * c) * 4 : kBufOff;
  }
  // rows of stage block sb (0 past the end: the ring's look-ahead then reads nothing)
  auto block_rows = [&](int64_t sb) -> uint32_t {
    return sb < stages ? static_cast<uint32_t>(min<int64_t>(C::R, p.rows - sb * C::R)) : 0u;
  };
  f32x4 raw[C::D][C::F], rawm[C::D][C::F];
  auto ring_load = [&](int64_t i, f32x4 (&a)[C::F], f32x4 (&m)[C::F]) {
    const int64_t sb = static_cast<int64_t>(bx) + i * nbx;
    const uint32_t nr = block_rows(sb);
    const int64_t r0 = (nr ? sb : 0) * C::R;
    const auto ra = buf_rsrc(p.A + r0 * p.lda, nr * static_cast<uint32_t>(p.lda) * 4);
#pragma unroll
    for (int u = 0; u < C::F; ++u) a[u] = buf_ld4(ra, aoff[u]);
    if constexpr (MASK) {
      const auto rm = buf_rsrc(p.mask + r0 * p.ldm, nr * static_cast<uint32_t>(p.ldm) * 4);
#pragma unroll
      for (int u = 0; u < C::F; ++u) m[u] = buf_ld4(rm, moff[u]);
    }
  };
  if (PW == 0 || producer) {
#pragma unroll
    for (int d = 0; d < C::D; ++d) ring_load(d, raw[d], rawm[d]);
  }

  // ---- W's slice → LDS (coalesced along whichever of k / n is contiguous in memory, scaled
  // there), then each wave's fragments (tile t = cg·NTW + tw, k step q, planes 0..2) → registers.
  // All loads of a kind are issued before any is used: a load under a runtime condition inside
  // an element loop made hipcc wait vmcnt(0) after each one.
  bf16x8 wf[NTW][KQ][3];
  f32x4 bias4[NTW];
  bool w_nk;  // W staged as [n][k] (else [k][n])
  {
    constexpr int NSL = 16 * NTS;                 // slice columns
    constexpr int LDW = NSL + 4;                  // [k][n] layout: padded row of k
    constexpr int LDK = C::K + ((8 - C::K) % 64 + 64) % 64;  // [n][k] layout: ≡ 8 dwords mod 64
    constexpr int EW = (C::K * NSL + C::THREADS - 1) / C::THREADS;
    static_assert(C::K * LDW * 4 <= C::LDS && NSL * LDK * 4 <= C::LDS,
                  "W staging must fit the kernel's LDS");
    float* sW = reinterpret_cast<float*>(x3s_smem);  // before the planes are used
    const bool kfast = p.bsk == 1;
    const bool vec = (reinterpret_cast<uintptr_t>(p.B) & 15) == 0 &&
                     (kfast ? p.bsn % 4 == 0 : (p.bsn == 1 && p.bsk % 4 == 0 && p.N % 4 == 0));
    // W contiguous along k (the forward's nn.Linear weight [N, K]): float4 pieces of a column
    // n stored as they are, sW[n][k] (16-byte writes, 8 consecutive lanes on 32 banks), and a
    // fragment is two 16-byte reads (LDK ≡ 8 mod 64: the 16 lanes of a ds_read_b128 group on
    // distinct banks). Otherwise sW[k][n] with scalar fragment reads.
    const bool nk = vec && kfast;
    w_nk = nk;
    if (vec) {
      // float4 pieces along the contiguous dimension, all in flight at once: one round trip
      // (8 pieces per thread at K = 128 and 128 columns)
      constexpr int E4 = C::K * NSL / 4;
      constexpr int EV = (E4 + C::THREADS - 1) / C::THREADS;
      f32x4 wv[EV];
      int ek[EV], en[EV];
#pragma unroll
      for (int r = 0; r < EV; ++r) {
        const int e = min(tid + C::THREADS * r, E4 - 1);
        ek[r] = kfast ? 4 * (e % (C::K / 4)) : e / (NSL / 4);
        en[r] = kfast ? e / (C::K / 4) : 4 * (e % (NSL / 4));
        const int n = n0 + en[r] < p.N ? n0 + en[r] : p.N - (kfast ? 1 : 4);
        wv[r] = ld4(p.B + static_cast<int64_t>(ek[r]) * p.bsk + static_cast<int64_t>(n) * p.bsn);
      }
      if (p.b_row_count) {
        f32x4 cnt[EV];
#pragma unroll
        for (int r = 0; r < EV; ++r) {
          if (kfast) {  // (the counts need not be 16-byte aligned)
            const float* cp = p.b_row_count + ek[r];
            cnt[r] = f32x4{cp[0], cp[1], cp[2], cp[3]};
          } else {
            const float c1 = p.b_row_count[ek[r]];
            cnt[r] = f32x4{c1, c1, c1, c1};
          }
        }
#pragma unroll
        for (int r = 0; r < EV; ++r)
#pragma unroll
          for (int j = 0; j < 4; ++j) wv[r][j] *= 1.f / fmaxf(cnt[r][j], 1.f);
      }
#pragma unroll
      for (int r = 0; r < EV; ++r) {
        f32x4 w = wv[r];
        if (p.b_scale != 0.f) w *= p.b_scale;
        if (n0 + en[r] >= p.N) w = f32x4{0.f, 0.f, 0.f, 0.f};
        if (tid + C::THREADS * r < E4) {
          float* dst = kfast ? sW + en[r] * LDK + ek[r] : sW + ek[r] * LDW + en[r];
          *reinterpret_cast<f32x4*>(dst) = w;
        }
      }
    } else {
      // any strides: chunks of 8 elements per thread, 8 loads in flight, sW[k][n]
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
          if (r0 + r < EW && tid + C::THREADS * (r0 + r) < C::K * NSL) sW[ek[r] * LDW + en[r]] = w;
        }
      }
    }
    __syncthreads();
  }

  // each computing wave's W fragments (tile t = cg·NTW + tw, k step q, planes 0..2) and bias
  auto load_w_frags = [&]() {
    constexpr int NSL = 16 * NTS;
    constexpr int LDW = NSL + 4;
    constexpr int LDK = C::K + ((8 - C::K) % 64 + 64) % 64;
    const float* sW = reinterpret_cast<const float*>(x3s_smem);
    const bool nk = w_nk;
#pragma unroll
    for (int tw = 0; tw < NTW; ++tw) {
      const int col = 16 * (cg * NTW + tw) + i16;
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        float v[8];
        if (nk) {
          const f32x4 lo4 = *reinterpret_cast<const f32x4*>(sW + col * LDK + 32 * q + 4 * g);
          const f32x4 hi4 = *reinterpret_cast<const f32x4*>(sW + col * LDK + 32 * q + 16 + 4 * g);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] = lo4[j];
            v[4 + j] = hi4[j];
          }
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            v[j] = sW[(32 * q + (j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4))) * LDW + col];
        }
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
  };

  const uint64_t drop_seed = p.drop_seed ? *p.drop_seed : 0ull;
  const uint32_t drop_thr = dropout_threshold(p.drop_keep);
  const uint64_t a_seed = p.a_drop_seed ? *p.a_drop_seed : 0ull;
  const uint32_t a_thr = dropout_threshold(p.a_drop_keep);

  // split stage s (its ring slot a / m) into plane buffer buf: input dropout, ReLU mask or
  // binarization, the three bf16 terms in MFMA-fragment order (+ row sums for row_inv)
  auto split_stage = [&](int64_t s, int buf, const f32x4 (&a)[C::F], const f32x4 (&m)[C::F]) {
    const int64_t r0 = (static_cast<int64_t>(bx) + s * nbx) * C::R;
    char* pb = planes + static_cast<size_t>(buf) * 3 * C::PLANE_BYTES;
#pragma unroll
    for (int u = 0; u < C::F; ++u) {
      const int f = stid + C::STHREADS * u;
      if (C::F4 % C::STHREADS != 0 && f >= C::F4) continue;
      const int rl = f / C::LPR, c = f % C::LPR;
      f32x4 x = a[u];
      const uint32_t e = static_cast<uint32_t>(r0 + rl) * static_cast<uint32_t>(C::K) + 4 * c;
      if constexpr (SPL == kSplDrop) {
        x = dropout_apply4(x, a_seed, e >> 2, a_thr, p.a_drop_scale);
      } else if constexpr (SPL == kSplAny) {
        if (p.a_drop_seed) x = dropout_apply4(x, a_seed, e >> 2, a_thr, p.a_drop_scale);
      }
      if constexpr (MASK) {
        x = relu_mask(x, m[u]);
      } else if constexpr (SPL == kSplAny) {
        if (p.binarize_a) {
#pragma unroll
          for (int cc = 0; cc < 4; ++cc) x[cc] = x[cc] > 0.f ? 1.f : 0.f;
        }
        if (p.row_inv) {
          float rs = (x.x + x.y) + (x.z + x.w);
#pragma unroll
          for (int o = 1; o < C::LPR; o <<= 1) rs += __shfl_xor(rs, o);
          if (c == 0) s_inv[buf * C::R + rl] = 1.f / fmaxf(rs, 1.f);
        }
      }
      bf16x4 h, md, lo;
      split3x4(x, h, md, lo);
      const int q = c >> 3, e8 = c & 7, gg = e8 & 3, half = e8 >> 2, j = rl & 15;
      const size_t off = (static_cast<size_t>(rl >> 4) * KQ + q) * 1024 +
                         static_cast<size_t>(gg * 16 + (j ^ (2 * gg + (q & 1)))) * 16 + half * 8;
      *reinterpret_cast<bf16x4*>(pb + off) = h;
      *reinterpret_cast<bf16x4*>(pb + C::PLANE_BYTES + off) = md;
      *reinterpret_cast<bf16x4*>(pb + 2 * C::PLANE_BYTES + off) = lo;
    }
  };

  // One pipeline step: stage i's planes (buffer i & 1) are complete after the barrier; its MFMAs
  // run, stage i + 1 is split from ring slot a / m into the other buffer and the slot refilled
  // with stage i + 1 + D, then stage i's epilogue. The split's vector work sits in the same
  // basic block as the MFMAs (SPL: no runtime branch in it), so the scheduler can interleave it
  // with the matrix instructions instead of running the two phases in turn.
  // consume(i, buf, mid): stage i's MFMAs from plane buffer buf, mid() (the cooperative form's
  // split of the next stage), then the epilogue
  auto consume = [&](int64_t i, int buf, auto&& mid) {
    const int64_t sb = static_cast<int64_t>(bx) + i * nbx;
    const int64_t r0 = sb * C::R;
    const uint32_t nr = block_rows(sb);
    const int64_t orow = r0 + 16 * rt + i16;
    const bool olive = orow < p.rows;
    // this lane's output pieces in the stage's Y / Y2 / res blocks (tiles past nt: no access)
    const uint32_t orl = 16 * rt + i16;
    uint32_t ocol[NTW];
#pragma unroll
    for (int tw = 0; tw < NTW; ++tw) {
      const int t = cg * NTW + tw;
      ocol[tw] = t < nt ? static_cast<uint32_t>(n0 + 16 * t + 4 * g) * 4 : kBufOff;
    }
    const auto ry = buf_rsrc(p.Y + r0 * p.ldy, nr * static_cast<uint32_t>(p.ldy) * 4);
    const uint32_t yo = orl * static_cast<uint32_t>(p.ldy) * 4;
    f32x4 ev[NTW];  // EPI 1: residual pieces, EPI 2: the Y pieces the product is added to
    if constexpr (EPI == kEpiRes) {
      const auto rr = buf_rsrc(p.res + r0 * p.ldres, nr * static_cast<uint32_t>(p.ldres) * 4);
      const uint32_t ro = orl * static_cast<uint32_t>(p.ldres) * 4;
#pragma unroll
      for (int tw = 0; tw < NTW; ++tw) ev[tw] = buf_ld4(rr, ro + ocol[tw]);
    } else if constexpr (EPI == kEpiAcc) {
#pragma unroll
      for (int tw = 0; tw < NTW; ++tw) ev[tw] = buf_ld4(ry, yo + ocol[tw]);
    }
    // the row scale before the MFMAs: the epilogue's first read of the accumulators then sits in
    // the same basic block as the last MFMA. With a branch in between, hipcc (ROCm 7.2) read the
    // accumulator registers without the MFMA→VALU wait states (stale results at NTW = 1, where
    // no second accumulation chain separates them)
    float inv = 1.f;
    if constexpr (!MASK && SPL == kSplAny) {
      if (p.row_inv) {
        inv = s_inv[buf * C::R + 16 * rt + i16];
        if (g == 0 && cg == 0 && n0 == 0 && olive) p.row_inv[orow] = inv;
      }
    }
    // MFMAs: this wave's row tile × column group, W in registers, stage i's fragments from LDS
    const char* fb = planes + static_cast<size_t>(buf) * 3 * C::PLANE_BYTES +
                     static_cast<size_t>(rt) * KQ * 1024;
    f32x4 acc[NTW];
#pragma unroll
    for (int tw = 0; tw < NTW; ++tw) acc[tw] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      const size_t so = static_cast<size_t>(q) * 1024 +
                        static_cast<size_t>(g * 16 + (i16 ^ (2 * g + (q & 1)))) * 16;
      const bf16x8 xh = *reinterpret_cast<const bf16x8*>(fb + so);
      const bf16x8 xm = *reinterpret_cast<const bf16x8*>(fb + C::PLANE_BYTES + so);
      const bf16x8 xl = *reinterpret_cast<const bf16x8*>(fb + 2 * C::PLANE_BYTES + so);
#pragma unroll
      for (int tw = 0; tw < NTW; ++tw)
        acc[tw] = mfma_x3(wf[tw][q][0], wf[tw][q][1], wf[tw][q][2], xh, xm, xl, acc[tw], false);
    }
    mid();
    // epilogue: lane (i16, g) holds row orow, columns n0 + 16t + 4g + 0..3; the scale and bias
    // unconditionally (inv = 1 without row_inv: bitwise the unscaled sum) and at once
    mfma_drain();
    f32x4 outv[NTW];
#pragma unroll
    for (int tw = 0; tw < NTW; ++tw) outv[tw] = acc[tw] * inv + bias4[tw];
    __amdgpu_buffer_rsrc_t ry2 = ry;
    uint32_t y2o = 0;
    if constexpr (EPI == kEpiRes) {
      ry2 = buf_rsrc(p.Y2 + r0 * p.ldy2, nr * static_cast<uint32_t>(p.ldy2) * 4);
      y2o = orl * static_cast<uint32_t>(p.ldy2) * 4;
    }
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
      if constexpr (EPI == kEpiAcc) v += ev[tw];
      buf_st4(ry, yo + ocol[tw], v);
      if constexpr (EPI == kEpiRes)
        buf_st4(ry2, y2o + ocol[tw], v + ev[tw]);
    }
  };
  // stages of this workgroup; stage s lives in ring slot s % D (static: D steps unrolled)
  const int64_t my_stages = bx < stages ? (stages - bx + nbx - 1) / nbx : 0;
  if (my_stages == 0) return;  // (uniform: no barrier below is reached by part of the workgroup)
  if constexpr (PW == 0) {
    load_w_frags();
    __syncthreads();  // the staging region becomes plane buffers
    split_stage(0, 0, raw[0], rawm[0]);
    ring_load(C::D, raw[0], rawm[0]);
    // One pipeline step: stage i's planes (buffer i & 1) are complete after the barrier; its MFMAs
    // run, stage i + 1 is split from ring slot a / m into the other buffer (its last reads, stage
    // i - 1's, were before the barrier) and the slot refilled with stage i + 1 + D, then stage
    // i's epilogue. The split's vector work sits in the same basic block as the MFMAs (SPL: no
    // runtime branch in it), so the scheduler can interleave it with the matrix instructions.
    auto step = [&](int64_t i, int buf, bool has_next, f32x4 (&a)[C::F], f32x4 (&m)[C::F]) {
      __syncthreads();
      consume(i, buf, [&]() {
        if (has_next) {
          split_stage(i + 1, buf ^ 1, a, m);
          ring_load(i + 1 + C::D, a, m);
        }
        // issue order: each MFMA followed by two vector instructions (the split's), which run
        // while the matrix core works (an MFMA holds vector issue for 8 of its 16 cycles)
#pragma unroll
        for (int k = 0; k < KQ * NTW * 6; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        }
      });
    };
    // Whole groups of D steps that all have a next stage run without a condition, the rest
    // after the loop: with a per-step condition inside the loop, the path that skipped steps left
    // the latest ring load last in the queue, and hipcc's merge at the loop header waited
    // vmcnt(0) — the whole ring drained once per group
    int64_t i0 = 0;
    for (; i0 + C::D < my_stages; i0 += C::D) {
#pragma unroll
      for (int d = 0; d < C::D; ++d)
        step(i0 + d, static_cast<int>((i0 + d) & 1), true, raw[(d + 1) % C::D],
             rawm[(d + 1) % C::D]);
    }
#pragma unroll
    for (int d = 0; d < C::D; ++d) {
      if (i0 + d < my_stages)
        step(i0 + d, static_cast<int>((i0 + d) & 1), i0 + d + 1 < my_stages, raw[(d + 1) % C::D],
             rawm[(d + 1) % C::D]);
    }
  } else if (producer) {
    // producers: stage i + 1 into the buffer the consumers left before this barrier
    __syncthreads();  // the consumers have their W fragments: the staging region is free
    split_stage(0, 0, raw[0], rawm[0]);
    ring_load(C::D, raw[0], rawm[0]);
    auto pstep = [&](int64_t i, bool has_next, f32x4 (&a)[C::F], f32x4 (&m)[C::F]) {
      __syncthreads();
      if (has_next) {
        split_stage(i + 1, static_cast<int>((i + 1) & 1), a, m);
        ring_load(i + 1 + C::D, a, m);
      }
    };
    int64_t i0 = 0;
    for (; i0 + C::D < my_stages; i0 += C::D) {
#pragma unroll
      for (int d = 0; d < C::D; ++d) pstep(i0 + d, true, raw[(d + 1) % C::D], rawm[(d + 1) % C::D]);
    }
#pragma unroll
    for (int d = 0; d < C::D; ++d) {
      if (i0 + d < my_stages)
        pstep(i0 + d, i0 + d + 1 < my_stages, raw[(d + 1) % C::D], rawm[(d + 1) % C::D]);
    }
  } else {
    // consumers: W fragments, then one stage per barrier
    load_w_frags();
    __syncthreads();
    for (int64_t i = 0; i < my_stages; ++i) {
      __syncthreads();
      consume(i, static_cast<int>(i & 1), []() {
        // fragment reads one k step ahead of the MFMAs (not all hoisted: registers)
        __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
#pragma unroll
        for (int q = 0; q < KQ; ++q) {
          if (q + 1 < KQ) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, NTW * 6, 0);
        }
      });
    }
  }
}
// One staged split-bf16 launch (k_row_gemm_x3s): persistent workgroups, at most one resident
// round, shared by a group's products in proportion to their rows; column slices XCD-paired.
template <int KQ, int NTW, int CG, bool MASK, int EPI, int SPL, int PW>
hgd_status launch_x3s(RowGemmGroup g, hipStream_t st, const char* fn) {
  constexpr int RT = (8 / CG) < (16 / KQ) ? (8 / CG) : (16 / KQ) >= 4 ? 4 : 2;
  using C = X3S<KQ, NTW, CG, RT, MASK, PW>;
  const void* kern = reinterpret_cast<const void*>(&k_row_gemm_x3s<KQ, NTW, CG, RT, MASK, EPI, SPL, PW>);
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
  hipLaunchKernelGGL((k_row_gemm_x3s<KQ, NTW, CG, RT, MASK, EPI, SPL, PW>), grid, dim3(C::THREADS), C::LDS,
                     st, g);
  return check_launch(fn);
}

// The split kind of a group: kSplPlain without the runtime flags, kSplDrop when every product has
// the input dropout and nothing else, kSplAny otherwise (branches; kSplDrop is instantiated only
// for the unmasked plain / residual epilogues, the ED-HNN lin_in forward)
int x3s_split_kind(const RowGemmGroup& g, int epi) {
  int flags = 0, drops = 0;
  for (int i = 0; i < g.count; ++i) {
    const RowGemm& q = g.p[i];
    flags += q.binarize_a || q.row_inv != nullptr;
    drops += q.a_drop_seed != nullptr;
  }
  if (flags == 0 && drops == 0) return kSplPlain;
  if (flags == 0 && drops == g.count && !g.p[0].mask && epi != kEpiAcc) return kSplDrop;
  return kSplAny;
}

template <int KQ, int NTW, int CG, int PW, bool MASK, int EPI>
hgd_status launch_x3s_spl(const RowGemmGroup& g, int spl, hipStream_t st, const char* fn) {
  if (spl == kSplPlain) return launch_x3s<KQ, NTW, CG, MASK, EPI, kSplPlain, PW>(g, st, fn);
  if constexpr (!MASK && EPI != kEpiAcc) {
    if (spl == kSplDrop) return launch_x3s<KQ, NTW, CG, MASK, EPI, kSplDrop, PW>(g, st, fn);
  }
  return launch_x3s<KQ, NTW, CG, MASK, EPI, kSplAny, PW>(g, st, fn);
}

template <int KQ, int NTW, int CG, int PW = 0>
hgd_status launch_x3s_epi(const RowGemmGroup& g, hipStream_t st, const char* fn) {
  // every product of a group has the same mask mode; the epilogue kind must match too
  const RowGemm& p = g.p[0];
  const int epi = p.Y2 ? kEpiRes : (p.accumulate ? kEpiAcc : kEpiPlain);
  for (int i = 1; i < g.count; ++i) {
    const RowGemm& q = g.p[i];
    HGD_REQUIRE((q.Y2 ? kEpiRes : (q.accumulate ? kEpiAcc : kEpiPlain)) == epi,
                "%s: grouped products need the same epilogue (residual / accumulate)", fn);
  }
  const int spl = x3s_split_kind(g, epi);
  if (p.mask) {
    if (epi == kEpiAcc) return launch_x3s_spl<KQ, NTW, CG, PW, true, kEpiAcc>(g, spl, st, fn);
    return launch_x3s_spl<KQ, NTW, CG, PW, true, kEpiPlain>(g, spl, st, fn);
  }
  if (epi == kEpiRes) return launch_x3s_spl<KQ, NTW, CG, PW, false, kEpiRes>(g, spl, st, fn);
  if (epi == kEpiAcc) return launch_x3s_spl<KQ, NTW, CG, PW, false, kEpiAcc>(g, spl, st, fn);
  return launch_x3s_spl<KQ, NTW, CG, PW, false, kEpiPlain>(g, spl, st, fn);
}

template <int KQ>
hgd_status launch_x3s_shape(const RowGemmGroup& g, int tiles, hipStream_t st, const char* fn) {
  const int nt = (std::min(g.p[0].N, 128) + 15) / 16;
  // default (measured at 144,242 × 128 and 69,716 / 31,668 × 64, profiles/r03_linear): one
  // tile per wave for the masked backward-data product, two tiles + producer waves otherwise
  if (tiles == 0) tiles = g.p[0].mask ? 1 : 3;
  if (tiles == 3 && nt > 2) {  // two tiles per wave + 4 producer waves
    if (nt <= 4) return launch_x3s_epi<KQ, 2, 2, 4>(g, st, fn);
    return launch_x3s_epi<KQ, 2, 4, 4>(g, st, fn);
  }
  if (tiles == 1 && nt > 2) {  // one column tile per wave, ≤ 128 registers: 2 workgroups per CU
    if (nt <= 4) return launch_x3s_epi<KQ, 1, 4>(g, st, fn);
    return launch_x3s_epi<KQ, 1, 8>(g, st, fn);
  }
  if (nt <= 1) return launch_x3s_epi<KQ, 1, 1>(g, st, fn);
  if (nt <= 2) return launch_x3s_epi<KQ, 2, 1>(g, st, fn);
  if (nt <= 4) return launch_x3s_epi<KQ, 2, 2>(g, st, fn);
  return launch_x3s_epi<KQ, 2, 4>(g, st, fn);
}

}  // namespace

template <>
hgd_status launch_x3s_k<HGD_X3S_KQ>(const RowGemmGroup& g, int tiles, hipStream_t st,
                                    const char* fn) {
  return launch_x3s_shape<HGD_X3S_KQ>(g, tiles, st, fn);
}

}  // namespace lin
}  // namespace hgd
