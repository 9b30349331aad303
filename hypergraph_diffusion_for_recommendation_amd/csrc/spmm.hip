// CSR row-gather SpMM hop for gfx950 (CDNA4, wave64).
//
// Replaces torch.sparse.mm(adj, X) / torch.sparse.mm(adj.t(), X) (HCCF.py:199, HGNN_HD4.py:459-462,
// HGCN.py:173-175) and the torch_scatter mean pair (layers2/EquivSetConv2.py:88-93) of the
// reference (paths relative to /root/reference/HD_SELFRec).
//
// Work mapping (HBM-bound gather, ~0.5 flop/B; no MFMA):
//   * one row of Y per group of G lanes; each lane owns VEC contiguous columns, so a group moves
//     one gathered X row per load instruction (d=64: G=16 lanes × float4 = 256 B, 4 rows per wave);
//   * the group loads G column indices (and weights) with one coalesced load and broadcasts them
//     with __shfl, then issues U independent row gathers before consuming any of them, so every
//     lane keeps U×16 B in flight (U=8: 8 KB per wave at d=64);
//   * the sum runs in edge order in fp32 (single accumulator, fmaf), so results are deterministic;
//   * rows longer than the split plan's threshold are cut into fixed-size chunks handled by extra
//     blocks placed FIRST in the grid (they are the longest work items); a fix-up kernel sums the
//     chunk partials in chunk order — no float atomics anywhere.
#include <cmath>

#include <hipcub/hipcub.hpp>

#include "device_util.h"
#include "hgd_internal.h"

namespace hgd {

struct SpmmArgs {
  const int64_t* rowptr;
  const int32_t* col;
  const float* val;
  const float* row_scale;
  int64_t row_begin, row_end;
  const float* X;
  int64_t ldx;
  float* Y;
  int64_t ldy;
  int32_t d;
  int32_t col0;  // first column handled by this launch (column passes for wide/odd d)
  int32_t epi;
  float slope;
  // split plan
  int64_t heavy_threshold;
  int64_t n_chunks;
  int64_t n_heavy;
  int32_t chunk;
  int32_t seg;  // 1: segmented short-row kernel (plan flag HGD_PLAN_SEGMENTED)
  const int32_t* chunk_heavy;
  const int32_t* heavy_rows;
  const int64_t* heavy_cptr;
  float* partial;  // [n_chunks, d]
  int64_t heavy_blocks;
  hgd_row_epilogue ex;  // used by the EX (hgd_spmm_fused) instantiations only
  // masked hop (hgd_spmm_masked, the MASK instantiations): the edge-dropped matrix of
  // SpAdjDropEdge as a view of its parent — edge e counts iff mask[e] != 0, with weight
  // val[e] / keep (IEEE, as the dropped COO's values)
  const uint8_t* mask;
  float keep;
  // 1 / keep when keep is a power of two (HCCF's 0.5), else 0: then w·inv_keep is w / keep bit
  // for bit (one exact real value, rounded once either way) at one multiply instead of the
  // IEEE division's ~10-instruction sequence per kept entry
  float inv_keep;
  int32_t mask_pair;  // two-batch masked walk (HGD_TUNE_MASK_PAIR)
  // XCD-interleaved column passes (HGD_TUNE_SPMM_PASS_INTERLEAVE): all n_pass column passes of a
  // wide row in ONE launch, the passes of a row block on consecutive workgroups of the same XCD
  int32_t n_pass;     // > 1: interleaved; else the launch covers the one pass at col0
  int32_t pass_cols;  // columns per pass when interleaved
  // source-blocked hop (hgd_spmm_blocked): a launch per source block k over the block-major
  // copy (hgd_spmm_col_blocks), whose rows of block k are a CSR of their own (rowptr =
  // blk_start + k·n_rows); with blk_accum the row adds s·Σ to the Y row the blocks before wrote
  int32_t blk_accum;
};

// vals[mask] / keepRate (HCCF.py:224)
__device__ __forceinline__ float scale_kept(const SpmmArgs& a, float w) {
  return a.inv_keep != 0.f ? w * a.inv_keep : __fdiv_rn(w, a.keep);
}

__device__ __forceinline__ float epilogue(float y, int epi, float slope) {
  if (epi == HGD_EPI_LEAKY_RELU) return y > 0.f ? y : y * slope;
  if (epi == HGD_EPI_RELU) return y > 0.f ? y : 0.f;
  return y;
}

// Cache-policy bits of the tuned variants (hgd_set_tuning(HGD_TUNE_SPMM_POLICY, bits)):
constexpr int kPolNtStore = 1;   // Y rows: non-temporal stores (written once, never re-read here)
constexpr int kPolNtIndex = 2;   // col / val streams: non-temporal loads (read exactly once)
constexpr int kPolNtGather = 4;  // gathered X rows: non-temporal loads
constexpr int kPolPrefetch = 8;  // software-pipelined index batches (see gather_sum)

// Scale, epilogue and store of one finished row r (all G lanes of the group call it together).
// With EX the hgd_row_epilogue runs in registers: the group holds the whole row (single column
// pass, checked on the host), so the LayerNorm statistics are two group_sum butterflies.
template <int G, int VEC, bool EX, bool NT_STORE>
__device__ __forceinline__ void finish_row(const SpmmArgs& a, int64_t r, float s, int l,
                                           int64_t coff, bool col_ok, float (&acc)[VEC]) {
  if constexpr (!EX) {
    if (a.blk_accum) {  // a later block of a column-blocked hop: Y = epi(s·Σ_block + Y)
      float prev[VEC];
      if (col_ok) {
        load_vec<VEC>(a.Y + r * a.ldy + coff, prev);
      } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) prev[i] = 0.f;
      }
#pragma unroll
      for (int i = 0; i < VEC; ++i) acc[i] = epilogue(acc[i] * s + prev[i], a.epi, a.slope);
      if (col_ok) store_vec<VEC, NT_STORE>(a.Y + r * a.ldy + coff, acc);
      return;
    }
  }
#pragma unroll
  for (int i = 0; i < VEC; ++i) acc[i] = epilogue(acc[i] * s, a.epi, a.slope);
  if constexpr (EX) {
    const hgd_row_epilogue& e = a.ex;
    if (e.act_out && col_ok) store_vec<VEC>(e.act_out + r * e.ld_act + coff, acc);
    if (e.layer_norm) {
      float t = 0.f;
      if (col_ok) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) t += acc[i];
      }
      const float mu = group_sum<G>(t) / static_cast<float>(a.d);
      t = 0.f;
      if (col_ok) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) t += (acc[i] - mu) * (acc[i] - mu);
      }
      const float rstd = 1.f / sqrtf(group_sum<G>(t) / static_cast<float>(a.d) + e.ln_eps);
      if (e.stats && l == 0) {
        e.stats[2 * r] = mu;
        e.stats[2 * r + 1] = rstd;
      }
      if (col_ok) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const float gm = e.ln_gamma ? e.ln_gamma[coff + i] : 1.f;
          const float bt = e.ln_beta ? e.ln_beta[coff + i] : 0.f;
          acc[i] = fmaf((acc[i] - mu) * rstd, gm, bt);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[i] *= e.out_scale;
    if (e.res1 && col_ok) {
      float rv[VEC];
      load_vec<VEC>(e.res1 + r * e.ld_res1 + coff, rv);
#pragma unroll
      for (int i = 0; i < VEC; ++i) acc[i] = fmaf(e.res1_scale, rv[i], acc[i]);
    }
    if (e.res2 && col_ok) {
      float rv[VEC];
      load_vec<VEC>(e.res2 + r * e.ld_res2 + coff, rv);
#pragma unroll
      for (int i = 0; i < VEC; ++i) acc[i] = fmaf(e.res2_scale, rv[i], acc[i]);
    }
  }
  if (col_ok) store_vec<VEC, NT_STORE>(a.Y + r * a.ldy + coff, acc);
  if constexpr (EX) {
    const hgd_row_epilogue& e = a.ex;
    if (e.sum_out && col_ok) {
      float rv[VEC];
      load_vec<VEC>(e.sum_res + r * e.ld_sum_res + coff, rv);
#pragma unroll
      for (int i = 0; i < VEC; ++i) rv[i] = acc[i] + rv[i];
      store_vec<VEC>(e.sum_out + r * e.ld_sum_out + coff, rv);
    }
  }
}

// Lane l's share of a batch of G column indices (and weights) starting at nonzero eb; with MASK
// also its keep flag (0 past the batch).
template <bool HAS_VAL, int POL, bool MASK = false>
__device__ __forceinline__ void load_index(const SpmmArgs& a, int64_t eb, int n, int l, int& c,
                                           float& w, int& keep) {
  c = 0;
  w = 1.f;
  keep = 0;
  if (l < n) {
    if constexpr (MASK) keep = a.mask[eb + l];
    if constexpr (POL & kPolNtIndex) {
      c = __builtin_nontemporal_load(a.col + eb + l);
      if constexpr (HAS_VAL) w = __builtin_nontemporal_load(a.val + eb + l);
    } else {
      c = a.col[eb + l];
      if constexpr (HAS_VAL) w = a.val[eb + l];
    }
  }
}

// Position of the j-th set bit (0-based) of a G-bit group mask: a popcount binary search.
template <int G>
__device__ __forceinline__ int nth_set_bit(unsigned long long m, int j) {
  int pos = 0;
#pragma unroll
  for (int w = G / 2; w >= 1; w >>= 1) {
    const int c = __popcll(m & ((1ull << w) - 1ull));
    if (j >= c) {
      j -= c;
      m >>= w;
      pos += w;
    }
  }
  return pos;
}

// MASK: packs the kept entries of a fetched batch to the front of the group (in edge order) with
// their weights val/keep; returns how many there are. Every lane of the group calls it.
template <int G, bool HAS_VAL>
__device__ __forceinline__ int compact_kept(const SpmmArgs& a, int l, int keep, int& c, float& w) {
  const unsigned long long bal = __ballot(keep != 0);
  const int base = (static_cast<int>(threadIdx.x) & 63) & ~(G - 1);
  const unsigned long long gm =
      G == 64 ? bal : (bal >> base) & ((1ull << (G == 64 ? 0 : G)) - 1ull);
  const int src = nth_set_bit<G>(gm, l);
  if constexpr (HAS_VAL) w = scale_kept(a, w);
  c = __shfl(c, src, G);
  if constexpr (HAS_VAL) w = __shfl(w, src, G);
  return __popcll(gm);
}

// The masked hop's walk (MASK): TWO index batches of G edges per step (2G edges, about G kept
// at keep = 0.5), their kept entries packed in edge order into 2G slots — slot j < G in lane j's
// register a, slot j >= G in lane j-G's register b — so a step gathers as many rows as an
// unmasked batch instead of half as many; the next pair of index batches is loaded before the
// gathers are issued. Sums in edge order: bitwise the one-batch walk and the compacted matrix's.
// PUSH (HGD_TUNE_MASK_PAIR = 2, the default): the packing is ONE forward permute per value and
// batch — each lane sends its entry to its slot (its rank among the kept entries of its batch,
// from a popcount of the lower lanes' keep bits; the dropped entries fill the slots after the
// kept ones, so every batch is a permutation of the group's lanes and no two lanes collide) —
// instead of every lane pulling its slot's entry after a binary search for the j-th set bit
// (nth_set_bit, three per step: ~4 dependent popcount rounds each). Same slots, same sums.
template <int G, int VEC, int U, bool HAS_VAL, int POL, bool PUSH>
__device__ __forceinline__ void gather_sum_mask2(const SpmmArgs& a, int64_t e0, int64_t e1,
                                                 int l, bool col_ok, float (&acc)[VEC],
                                                 int32_t col0) {
#pragma unroll
  for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
  const int64_t coff = static_cast<int64_t>(col0) + static_cast<int64_t>(l) * VEC;
  const int base = (static_cast<int>(threadIdx.x) & 63) & ~(G - 1);
  auto group_bits = [&](int keep) {
    const unsigned long long bal = __ballot(keep != 0);
    return G == 64 ? bal : (bal >> base) & ((1ull << (G == 64 ? 0 : G)) - 1ull);
  };
  auto load2 = [&](int64_t eb, int& c1, float& w1, int& k1, int& c2, float& w2, int& k2) {
    load_index<HAS_VAL, POL, true>(a, eb, static_cast<int>(min(static_cast<int64_t>(G), e1 - eb)),
                                   l, c1, w1, k1);
    const int64_t eb2 = eb + G;
    if (eb2 < e1) {
      load_index<HAS_VAL, POL, true>(
          a, eb2, static_cast<int>(min(static_cast<int64_t>(G), e1 - eb2)), l, c2, w2, k2);
    } else {
      c2 = 0;
      w2 = 1.f;
      k2 = 0;
    }
  };
  int nc1 = 0, nk1 = 0, nc2 = 0, nk2 = 0;
  float nw1 = 1.f, nw2 = 1.f;
  if (e0 < e1) load2(e0, nc1, nw1, nk1, nc2, nw2, nk2);
  for (int64_t eb = e0; eb < e1; eb += 2 * G) {
    const int c1 = nc1, k1 = nk1, c2 = nc2, k2 = nk2;
    const float w1 = nw1, w2 = nw2;
    if (eb + 2 * G < e1) load2(eb + 2 * G, nc1, nw1, nk1, nc2, nw2, nk2);
    const unsigned long long gm1 = group_bits(k1), gm2 = group_bits(k2);
    const int n1 = __popcll(gm1), n2 = __popcll(gm2), n = n1 + n2;
    if (n == 0) continue;  // group-uniform
    // slot l (register a) and slot l + G (register b) of the packed pair
    int ca, cb;
    float wa = 1.f, wb = 1.f;
    if constexpr (PUSH) {
      const unsigned long long below = (1ull << l) - 1ull;  // the group's lanes below l
      const int r1 = __popcll(gm1 & below), r2 = __popcll(gm2 & below);
      // batch 1 → slots [0, G) of register a; batch 2 → slot n1 + rank, i.e. register a of lane
      // (n1 + rank) for slots < G and register b of lane (n1 + rank − G) beyond: one permute
      // modulo G serves both, and each lane's a / b pick (l < n1) is the pull form's
      const int d1 = k1 ? r1 : n1 + (l - r1);
      const int d2 = ((k2 ? r2 : n2 + (l - r2)) + n1) & (G - 1);
      const int a1 = 4 * (base + d1), a2 = 4 * (base + d2);
      const int x1 = __builtin_amdgcn_ds_permute(a1, c1);
      const int x2 = __builtin_amdgcn_ds_permute(a2, c2);
      ca = l < n1 ? x1 : x2;
      cb = x2;
      if constexpr (HAS_VAL) {
        // vals[mask] / keepRate (HCCF.py:224), divided before the move (same IEEE quotient)
        const float v1 = scale_kept(a, w1), v2 = scale_kept(a, w2);
        const float y1 = __int_as_float(__builtin_amdgcn_ds_permute(a1, __float_as_int(v1)));
        const float y2 = __int_as_float(__builtin_amdgcn_ds_permute(a2, __float_as_int(v2)));
        wa = l < n1 ? y1 : y2;
        wb = y2;
      }
    } else {
      const int s1 = nth_set_bit<G>(gm1, l);
      const int s2a = nth_set_bit<G>(gm2, l >= n1 ? l - n1 : 0);
      const int s2b = nth_set_bit<G>(gm2, l + G - n1 < G ? l + G - n1 : 0);
      const int ca1 = __shfl(c1, s1, G), ca2 = __shfl(c2, s2a, G);
      cb = __shfl(c2, s2b, G);
      ca = l < n1 ? ca1 : ca2;
      if constexpr (HAS_VAL) {
        const float wa1 = __shfl(w1, s1, G), wa2 = __shfl(w2, s2a, G);
        wa = scale_kept(a, l < n1 ? wa1 : wa2);
        wb = scale_kept(a, __shfl(w2, s2b, G));
      }
    }
    for (int k = 0; k < n; k += U) {
      const bool hi = k >= G;  // group-uniform: U divides G, so a step stays in one register
      float xv[U][VEC];
      float w[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int kk = k + u;
        const int c = __shfl(hi ? cb : ca, kk & (G - 1), G);
        if constexpr (HAS_VAL) w[u] = __shfl(hi ? wb : wa, kk & (G - 1), G);
        if (kk < n && col_ok) {
          load_vec<VEC, (POL & kPolNtGather) != 0>(a.X + static_cast<int64_t>(c) * a.ldx + coff,
                                                   xv[u]);
        } else {
#pragma unroll
          for (int i = 0; i < VEC; ++i) xv[u][i] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (k + u < n) {
#pragma unroll
          for (int i = 0; i < VEC; ++i) {
            if constexpr (HAS_VAL)
              acc[i] = fmaf(w[u], xv[u][i], acc[i]);
            else
              acc[i] += xv[u][i];
          }
        }
      }
    }
  }
}

// Σ_{e in [e0,e1)} val[e] * X[col[e], cols of this lane], in edge order. With kPolPrefetch the
// index batch b+1 is loaded before the gathers of batch b are issued, so the dependent
// index → gather round trip is paid once per row instead of once per batch of G nonzeros.
// With MASK only the kept edges are summed (same order as over the compacted matrix).
template <int G, int VEC, int U, bool HAS_VAL, int POL, bool MASK = false>
__device__ __forceinline__ void gather_sum(const SpmmArgs& a, int64_t e0, int64_t e1, int l,
                                           bool col_ok, float (&acc)[VEC], int32_t col0) {
#pragma unroll
  for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
  const int64_t coff = static_cast<int64_t>(col0) + static_cast<int64_t>(l) * VEC;
  constexpr bool PF = (POL & kPolPrefetch) != 0;
  int nxc = 0, nxk = 0;
  float nxw = 1.f;
  if constexpr (PF) {
    if (e0 < e1)
      load_index<HAS_VAL, POL, MASK>(
          a, e0, static_cast<int>(min(static_cast<int64_t>(G), e1 - e0)), l, nxc, nxw, nxk);
  }
  for (int64_t eb = e0; eb < e1; eb += G) {
    int n = static_cast<int>(min(static_cast<int64_t>(G), e1 - eb));
    int myc, myk;
    float myw;
    if constexpr (PF) {
      myc = nxc;
      myw = nxw;
      myk = nxk;
      const int64_t en = eb + G;
      if (en < e1)
        load_index<HAS_VAL, POL, MASK>(
            a, en, static_cast<int>(min(static_cast<int64_t>(G), e1 - en)), l, nxc, nxw, nxk);
    } else {
      load_index<HAS_VAL, POL, MASK>(a, eb, n, l, myc, myw, myk);
    }
    if constexpr (MASK) n = compact_kept<G, HAS_VAL>(a, l, myk, myc, myw);
    for (int k = 0; k < n; k += U) {
      float xv[U][VEC];
      float w[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int kk = k + u;
        const int c = (G == 1) ? myc : __shfl(myc, kk, G);
        if constexpr (HAS_VAL) w[u] = (G == 1) ? myw : __shfl(myw, kk, G);
        if (kk < n && col_ok) {
          load_vec<VEC, (POL & kPolNtGather) != 0>(a.X + static_cast<int64_t>(c) * a.ldx + coff,
                                                   xv[u]);
        } else {
#pragma unroll
          for (int i = 0; i < VEC; ++i) xv[u][i] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (k + u < n) {
#pragma unroll
          for (int i = 0; i < VEC; ++i) {
            if constexpr (HAS_VAL)
              acc[i] = fmaf(w[u], xv[u][i], acc[i]);
            else
              acc[i] += xv[u][i];
          }
        }
      }
    }
  }
}

int g_mask_pair = 2;  // HGD_TUNE_MASK_PAIR: the masked hop walks two index batches per step
int g_mask_div = 0;   // HGD_TUNE_MASK_DIV: 1 = divide by keep even when it is a power of two

// MASK with G >= 8 lanes (U | G): the two-batch masked walk unless HGD_TUNE_MASK_PAIR is 0.
template <int G, int VEC, int U, bool HAS_VAL, int POL, bool MASK>
__device__ __forceinline__ void masked_or_plain_sum(const SpmmArgs& a, int64_t e0, int64_t e1,
                                                    int l, bool col_ok, float (&acc)[VEC],
                                                    int32_t col0) {
  if constexpr (MASK && G >= 8 && G % U == 0) {
    if (a.mask_pair == 2) {
      gather_sum_mask2<G, VEC, U, HAS_VAL, POL, true>(a, e0, e1, l, col_ok, acc, col0);
      return;
    }
    if (a.mask_pair) {
      gather_sum_mask2<G, VEC, U, HAS_VAL, POL, false>(a, e0, e1, l, col_ok, acc, col0);
      return;
    }
  }
  gather_sum<G, VEC, U, HAS_VAL, POL, MASK>(a, e0, e1, l, col_ok, acc, col0);
}

template <int G, int VEC, int U, bool HAS_VAL, int POL, bool EX, bool MASK = false>
__global__ __launch_bounds__(kBlock) void spmm_kernel(SpmmArgs a) {
  constexpr int GPB = kBlock / G;
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  int64_t bid = static_cast<int64_t>(blockIdx.x) - a.heavy_blocks;
  int32_t col0 = a.col0;
  if (a.n_pass > 1) {
    // workgroups are dispatched to the 8 XCDs round-robin (blockIdx mod 8): the n_pass passes of
    // row block (k / n_pass)·8 + x run back to back on XCD x, so the later passes find the row
    // pointers and index stream in that XCD's L2 and fetch the other quarters of the same
    // gathered rows while the DRAM pages are open (no split rows here: heavy_blocks is 0)
    const int64_t x = bid & 7, k = bid >> 3;
    col0 = static_cast<int32_t>((k % a.n_pass) * a.pass_cols);
    bid = (k / a.n_pass) * 8 + x;
  }
  const int64_t coff = static_cast<int64_t>(col0) + static_cast<int64_t>(l) * VEC;
  const bool col_ok = coff < a.d;
  float acc[VEC];

  if (bid < 0) {
    const int64_t t = static_cast<int64_t>(blockIdx.x) * GPB + g;
    if (t >= a.n_chunks) return;
    const int h = a.chunk_heavy[t];
    const int64_t r = a.heavy_rows[h];
    if (r < a.row_begin || r >= a.row_end) return;
    const int64_t k = t - a.heavy_cptr[h];
    const int64_t re = a.rowptr[r + 1];
    const int64_t e0 = a.rowptr[r] + k * a.chunk;
    const int64_t e1 = min(e0 + static_cast<int64_t>(a.chunk), re);
    masked_or_plain_sum<G, VEC, U, HAS_VAL, POL, MASK>(a, e0, e1, l, col_ok, acc, col0);
    if (col_ok) store_vec<VEC>(a.partial + t * a.d + coff, acc);
    return;
  }

  const int64_t r = a.row_begin + bid * GPB + g;
  if (r >= a.row_end) return;
  const int64_t e0 = a.rowptr[r];
  const int64_t e1 = a.rowptr[r + 1];
  if (a.heavy_threshold > 0 && e1 - e0 > a.heavy_threshold) return;  // split-plan row
  masked_or_plain_sum<G, VEC, U, HAS_VAL, POL, MASK>(a, e0, e1, l, col_ok, acc, col0);
  const float s = a.row_scale ? a.row_scale[r] : 1.f;
  finish_row<G, VEC, EX, (POL & kPolNtStore) != 0>(a, r, s, l, coff, col_ok, acc);
}

// Segmented variant for short rows (hgd_split_plan.flags & HGD_PLAN_SEGMENTED): a group owns
// G consecutive rows and walks their nonzeros as ONE flat stream [rowptr[r0], rowptr[r0+G]) in
// batches of G indices, so every gather batch is full whatever the row lengths, the row pointers
// and row scales of all G rows arrive in one coalesced load, and the accumulator is flushed
// (scale, epilogue, store) at each row boundary. Sums stay in edge order per row.
template <int G, int VEC, int U, bool HAS_VAL, int POL, bool EX>
__global__ __launch_bounds__(kBlock) void spmm_seg_kernel(SpmmArgs a) {
  constexpr int GPB = kBlock / G;
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  const int64_t r0 = a.row_begin + (static_cast<int64_t>(blockIdx.x) * GPB + g) * G;
  if (r0 >= a.row_end) return;
  const int nr = static_cast<int>(min(static_cast<int64_t>(G), a.row_end - r0));
  int64_t my_end = 0;  // lane j: end of local row j
  float my_s = 1.f;    // lane j: scale of local row j
  if (l < nr) {
    my_end = a.rowptr[r0 + l + 1];
    if (a.row_scale) my_s = a.row_scale[r0 + l];
  }
  const int64_t e_begin = a.rowptr[r0];
  const int64_t e_end = __shfl(my_end, nr - 1, G);
  const int64_t coff = static_cast<int64_t>(a.col0) + static_cast<int64_t>(l) * VEC;
  const bool col_ok = coff < a.d;
  float acc[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
  int cur = 0;
  int64_t next_b = __shfl(my_end, 0, G);

  auto flush = [&]() {
    const float s = __shfl(my_s, cur, G);
    float y[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      y[i] = acc[i];
      acc[i] = 0.f;
    }
    finish_row<G, VEC, EX, (POL & kPolNtStore) != 0>(a, r0 + cur, s, l, coff, col_ok, y);
    ++cur;
    const int64_t nb = __shfl(my_end, cur < nr ? cur : 0, G);
    next_b = cur < nr ? nb : INT64_MAX;
  };

  constexpr bool PF = (POL & kPolPrefetch) != 0;
  int nxc = 0, unused_keep = 0;
  float nxw = 1.f;
  if constexpr (PF) {
    if (e_begin < e_end)
      load_index<HAS_VAL, POL>(
          a, e_begin, static_cast<int>(min(static_cast<int64_t>(G), e_end - e_begin)), l, nxc,
          nxw, unused_keep);
  }
  for (int64_t eb = e_begin; eb < e_end; eb += G) {
    const int n = static_cast<int>(min(static_cast<int64_t>(G), e_end - eb));
    int myc;
    float myw;
    if constexpr (PF) {
      myc = nxc;
      myw = nxw;
      const int64_t en = eb + G;
      if (en < e_end)
        load_index<HAS_VAL, POL>(
            a, en, static_cast<int>(min(static_cast<int64_t>(G), e_end - en)), l, nxc, nxw,
            unused_keep);
    } else {
      load_index<HAS_VAL, POL>(a, eb, n, l, myc, myw, unused_keep);
    }
    for (int k = 0; k < n; k += U) {
      float xv[U][VEC];
      float w[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int kk = k + u;
        const int c = __shfl(myc, kk, G);
        if constexpr (HAS_VAL) w[u] = __shfl(myw, kk, G);
        if (kk < n && col_ok) {
          load_vec<VEC, (POL & kPolNtGather) != 0>(a.X + static_cast<int64_t>(c) * a.ldx + coff,
                                                   xv[u]);
        } else {
#pragma unroll
          for (int i = 0; i < VEC; ++i) xv[u][i] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (k + u < n) {
          const int64_t e = eb + k + u;
          while (e >= next_b) flush();  // group-uniform; also emits empty rows
#pragma unroll
          for (int i = 0; i < VEC; ++i) {
            if constexpr (HAS_VAL)
              acc[i] = fmaf(w[u], xv[u][i], acc[i]);
            else
              acc[i] += xv[u][i];
          }
        }
      }
    }
  }
  while (cur < nr) flush();
}

// One block per split row: each of the GPB lane groups sums the chunk partials
// t = first + g, first + g + GPB, ... (FU independent loads in flight), then group 0 adds the
// GPB group sums in group order. The combine order is fixed by (chunk count, GPB), so the result
// is deterministic run to run; a popular item with ~10^4 chunks is reduced by GPB·FU loads in
// flight instead of one serial chain.
template <int G, int VEC, bool EX>
__global__ __launch_bounds__(kBlock) void spmm_fixup_kernel(SpmmArgs a) {
  constexpr int GPB = kBlock / G;
  constexpr int FU = 4;
  __shared__ float s_acc[GPB][G * VEC];
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  const int64_t h = blockIdx.x;
  const int64_t r = a.heavy_rows[h];
  if (r < a.row_begin || r >= a.row_end) return;  // block-uniform
  const int64_t coff = static_cast<int64_t>(a.col0) + static_cast<int64_t>(l) * VEC;
  const bool col_ok = coff < a.d;
  float acc[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
  const int64_t t0 = a.heavy_cptr[h], t1 = a.heavy_cptr[h + 1];
  for (int64_t t = t0 + g; t < t1; t += GPB * FU) {
    float v[FU][VEC];
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      const int64_t tt = t + static_cast<int64_t>(u) * GPB;
      if (tt < t1 && col_ok) {
        load_vec<VEC>(a.partial + tt * a.d + coff, v[u]);
      } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) v[u][i] = 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < FU; ++u)
#pragma unroll
      for (int i = 0; i < VEC; ++i) acc[i] += v[u][i];
  }
#pragma unroll
  for (int i = 0; i < VEC; ++i) s_acc[g][l * VEC + i] = acc[i];
  __syncthreads();
  if (g != 0) return;  // group 0 (all of its lanes: finish_row reduces over the group)
#pragma unroll
  for (int i = 0; i < VEC; ++i) acc[i] = s_acc[0][l * VEC + i];
  for (int k = 1; k < GPB; ++k)
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[i] += s_acc[k][l * VEC + i];
  const float s = a.row_scale ? a.row_scale[r] : 1.f;
  finish_row<G, VEC, EX, false>(a, r, s, l, coff, col_ok, acc);
}

namespace {

// Tuning knobs (hgd_set_tuning); defaults are the measured best on MI355X.
constexpr int kDefaultPolicy = kPolPrefetch;
int g_unroll = 8;
int g_policy = kDefaultPolicy;
// widest column pass of the float4 path without a fused epilogue; 0 = auto: rows up to 128
// floats in one pass, wider rows in 64-column passes (measured on MI355X at 100 M edges, d = 256:
// 64-column passes 64.9 ms per fwd+bwd, 128: 66.3 ms, one 256-wide pass of 64 lanes: 69.4 ms)
int g_pass_cols = 0;
// HGD_TUNE_SPMM_PASS_INTERLEAVE: 1 = a wide row's column passes as ONE launch, interleaved so the
// passes of a row block run back to back on one XCD (see spmm_kernel); 0 = a launch per pass
int g_pass_interleave = 0;
// HGD_TUNE_SPMM_BLOCKED_SEG: 1 = the source-blocked hop walks each block's short rows with the
// segmented kernel (a group owns G consecutive rows as one nonzero stream); 0 = a row per group
int g_blocked_seg = 0;

template <int G, int VEC, int U, int POL, bool EX = false>
void launch_kernel(const SpmmArgs& a, bool has_val, bool seg, int64_t blocks, hipStream_t st) {
  if constexpr (POL == kDefaultPolicy && U == 8) {
    if (a.mask) {  // masked (edge-dropped view) hop: the row kernel only
      if (has_val)
        hipLaunchKernelGGL((spmm_kernel<G, VEC, U, true, POL, EX, true>), dim3(blocks),
                           dim3(kBlock), 0, st, a);
      else
        hipLaunchKernelGGL((spmm_kernel<G, VEC, U, false, POL, EX, true>), dim3(blocks),
                           dim3(kBlock), 0, st, a);
      return;
    }
  }
  if constexpr (G >= 8) {
    if (seg) {
      if (has_val)
        hipLaunchKernelGGL((spmm_seg_kernel<G, VEC, U, true, POL, EX>), dim3(blocks),
                           dim3(kBlock), 0, st, a);
      else
        hipLaunchKernelGGL((spmm_seg_kernel<G, VEC, U, false, POL, EX>), dim3(blocks),
                           dim3(kBlock), 0, st, a);
      return;
    }
  }
  if (has_val)
    hipLaunchKernelGGL((spmm_kernel<G, VEC, U, true, POL, EX>), dim3(blocks), dim3(kBlock), 0,
                       st, a);
  else
    hipLaunchKernelGGL((spmm_kernel<G, VEC, U, false, POL, EX>), dim3(blocks), dim3(kBlock), 0,
                       st, a);
}

template <int G, int VEC, bool EX>
void launch_tuned(const SpmmArgs& a, bool has_val, bool seg, int64_t blocks, hipStream_t st) {
  if (a.mask) {
    launch_kernel<G, VEC, 8, kDefaultPolicy, EX>(a, has_val, false, blocks, st);
  } else if constexpr (EX) {
    launch_kernel<G, VEC, 8, kDefaultPolicy, true>(a, has_val, seg, blocks, st);
  } else if constexpr (G == 16 && VEC == 4) {
    // the d = 64 path carries the tuning matrix (unroll × {plain, nt-store, prefetch, both,
    // prefetch + nt-index, prefetch + nt-index + nt-store})
#define HGD_POL_CASES(U)                                                            \
    switch (g_policy) {                                                             \
      case 0: return launch_kernel<G, VEC, U, 0>(a, has_val, seg, blocks, st);      \
      case 1: return launch_kernel<G, VEC, U, 1>(a, has_val, seg, blocks, st);      \
      case 9: return launch_kernel<G, VEC, U, 9>(a, has_val, seg, blocks, st);      \
      case 10: return launch_kernel<G, VEC, U, 10>(a, has_val, seg, blocks, st);    \
      case 11: return launch_kernel<G, VEC, U, 11>(a, has_val, seg, blocks, st);    \
      default: return launch_kernel<G, VEC, U, 8>(a, has_val, seg, blocks, st);     \
    }
    if (g_unroll >= 16) { HGD_POL_CASES(16) }
    HGD_POL_CASES(8)
#undef HGD_POL_CASES
  } else {
    launch_kernel<G, VEC, 8, kDefaultPolicy>(a, has_val, seg, blocks, st);
  }
}

template <int G, int VEC, bool EX>
hgd_status launch_g(SpmmArgs a, bool has_val, hipStream_t st) {
  constexpr int GPB = kBlock / G;
  const int64_t rows = a.row_end - a.row_begin;
  if constexpr (G >= 8) {
    if (a.seg) {
      const int64_t sblocks = (rows + static_cast<int64_t>(GPB) * G - 1) / (GPB * G);
      if (sblocks <= 0) return HGD_OK;
      if (sblocks > 0x7fffffffLL) return fail(HGD_ERR_UNSUPPORTED, "hgd_spmm: grid too large");
      launch_tuned<G, VEC, EX>(a, has_val, true, sblocks, st);
      return check_launch("hgd_spmm segmented kernel");
    }
  }
  int64_t light_blocks = (rows + GPB - 1) / GPB;
  a.heavy_blocks = (a.n_chunks + GPB - 1) / GPB;
  if (a.n_pass > 1) light_blocks = (light_blocks + 7) / 8 * 8 * a.n_pass;  // (no split rows)
  const int64_t blocks = light_blocks + a.heavy_blocks;
  if (blocks > 0) {
    if (blocks > 0x7fffffffLL) return fail(HGD_ERR_UNSUPPORTED, "hgd_spmm: grid too large");
    launch_tuned<G, VEC, EX>(a, has_val, false, blocks, st);
    hgd_status s = check_launch("hgd_spmm kernel");
    if (s != HGD_OK) return s;
  }
  if (a.n_heavy > 0) {
    if (a.n_heavy > 0x7fffffffLL) return fail(HGD_ERR_UNSUPPORTED, "hgd_spmm: too many split rows");
    hipLaunchKernelGGL((spmm_fixup_kernel<G, VEC, EX>), dim3(a.n_heavy), dim3(kBlock), 0, st,
                       a);
    return check_launch("hgd_spmm fixup");
  }
  return HGD_OK;
}

template <int VEC, bool EX = false>
hgd_status launch_vec(int G, const SpmmArgs& a, bool has_val, hipStream_t st) {
  switch (G) {
    case 1: return launch_g<1, VEC, EX>(a, has_val, st);
    case 2: return launch_g<2, VEC, EX>(a, has_val, st);
    case 4: return launch_g<4, VEC, EX>(a, has_val, st);
    case 8: return launch_g<8, VEC, EX>(a, has_val, st);
    case 16: return launch_g<16, VEC, EX>(a, has_val, st);
    case 32: return launch_g<32, VEC, EX>(a, has_val, st);
    case 64: return launch_g<64, VEC, EX>(a, has_val, st);
    default: return fail(HGD_ERR_UNSUPPORTED, "hgd_spmm: unsupported group size %d", G);
  }
}

}  // namespace
}  // namespace hgd

extern "C" size_t hgd_spmm_workspace_size(const hgd_split_plan* plan, int32_t d) {
  if (!plan || plan->n_heavy <= 0 || plan->threshold <= 0 || d <= 0) return 0;
  return hgd::align_up(static_cast<size_t>(plan->n_chunks) * static_cast<size_t>(d) * 4);
}

namespace hgd {
namespace {

hgd_status spmm_impl(const int64_t* rowptr, const int32_t* col, const float* val,
                     const float* row_scale, int64_t n_rows, int64_t n_src_rows, int64_t row_begin,
                     int64_t row_end, const float* X, int64_t ldx, float* Y, int64_t ldy,
                     int32_t d, int32_t epilogue, float slope, const hgd_row_epilogue* ex,
                     const uint8_t* mask, float keep, const hgd_split_plan* plan,
                     void* workspace, size_t workspace_bytes, void* stream, const char* fn,
                     const int64_t* blk_seg = nullptr, int32_t n_blk = 0) {
  // blk_seg (hgd_spmm_blocked): the block-major blk_start (rowptr is the same pointer), col / val
  // the block-major arrays
  HGD_REQUIRE(d > 0, "%s: d must be > 0 (got %d)", fn, d);
  HGD_REQUIRE(n_rows >= 0 && n_src_rows >= 0, "%s: negative sizes", fn);
  HGD_REQUIRE(row_begin >= 0 && row_begin <= row_end && row_end <= n_rows,
              "%s: row range [%lld,%lld) outside [0,%lld)", fn, (long long)row_begin,
              (long long)row_end, (long long)n_rows);
  HGD_REQUIRE(ldx >= d && ldy >= d, "%s: ldx/ldy must be >= d", fn);
  HGD_REQUIRE(epilogue >= HGD_EPI_NONE && epilogue <= HGD_EPI_RELU, "%s: bad epilogue %d", fn,
              epilogue);
  if (ex) {
    HGD_REQUIRE(epilogue == HGD_EPI_NONE || slope >= 0.f,
                "%s: a fused activation needs slope >= 0 (got %g)", fn, (double)slope);
    HGD_REQUIRE(ex->layer_norm == 0 || ex->layer_norm == 1, "%s: layer_norm must be 0/1", fn);
    HGD_REQUIRE(!ex->res1 || ex->ld_res1 >= d, "%s: ld_res1 < d", fn);
    HGD_REQUIRE(!ex->res2 || ex->ld_res2 >= d, "%s: ld_res2 < d", fn);
    HGD_REQUIRE(!ex->act_out || ex->ld_act >= d, "%s: ld_act < d", fn);
    HGD_REQUIRE((ex->sum_out == nullptr) == (ex->sum_res == nullptr),
                "%s: sum_out and sum_res go together", fn);
    HGD_REQUIRE(!ex->sum_out || (ex->ld_sum_out >= d && ex->ld_sum_res >= d),
                "%s: ld_sum_out / ld_sum_res < d", fn);
  }
  if (row_end == row_begin) return HGD_OK;
  // col / X may be NULL for a structure without nonzeros (never dereferenced then).
  HGD_REQUIRE(rowptr && Y, "%s: null rowptr/Y", fn);
  HGD_REQUIRE(X || n_src_rows == 0, "%s: null X", fn);

  SpmmArgs a{};
  a.rowptr = rowptr;
  a.col = col;
  a.val = val;
  a.row_scale = row_scale;
  a.row_begin = row_begin;
  a.row_end = row_end;
  a.X = X;
  a.ldx = ldx;
  a.Y = Y;
  a.ldy = ldy;
  a.d = d;
  a.epi = epilogue;
  a.slope = slope;
  if (ex) a.ex = *ex;
  a.mask = mask;
  a.keep = keep;
  {
    int e2 = 0;
    a.inv_keep = (!g_mask_div && keep > 0.f && std::frexp(keep, &e2) == 0.5f) ? 1.f / keep : 0.f;
  }
  a.mask_pair = g_mask_pair;
  if (plan && plan->threshold > 0 && plan->n_heavy > 0) {
    HGD_REQUIRE(plan->chunk > 0 && plan->heavy_rows && plan->heavy_cptr && plan->chunk_heavy,
                "%s: incomplete split plan", fn);
    const size_t need = hgd_spmm_workspace_size(plan, d);
    if (workspace_bytes < need || (need && !workspace))
      return fail(HGD_ERR_WORKSPACE, "%s: workspace %zu < required %zu", fn, workspace_bytes,
                  need);
    a.heavy_threshold = plan->threshold;
    a.chunk = plan->chunk;
    a.n_chunks = plan->n_chunks;
    a.n_heavy = plan->n_heavy;
    a.chunk_heavy = plan->chunk_heavy;
    a.heavy_rows = plan->heavy_rows;
    a.heavy_cptr = plan->heavy_cptr;
    a.partial = static_cast<float*>(workspace);
  } else if (plan && (plan->flags & HGD_PLAN_SEGMENTED) && !mask) {
    a.seg = 1;  // only without split rows: the segmented walk covers every nonzero of its rows
  }

  hipStream_t st = as_stream(stream);
  const bool has_val = val != nullptr;
  auto al16 = [](const void* p, int64_t ld) {
    return p == nullptr || (reinterpret_cast<uintptr_t>(p) % 16 == 0 && ld % 4 == 0);
  };
  bool aligned = al16(X, ldx) && al16(Y, ldy) && (d % 4 == 0);
  if (ex)
    aligned = aligned && al16(ex->res1, ex->ld_res1) && al16(ex->res2, ex->ld_res2) &&
              al16(ex->act_out, ex->ld_act) && al16(ex->sum_out, ex->ld_sum_out) &&
              al16(ex->sum_res, ex->ld_sum_res);
  if (ex && ex->layer_norm && (aligned ? d > 256 : d > 64))
    return fail(HGD_ERR_UNSUPPORTED,
                "%s: layer_norm needs d <= 256 (16-byte aligned rows) or d <= 64 (got d=%d%s)",
                fn, d, aligned ? "" : ", unaligned");
  if (aligned) {
    // float4 path: one pass when d/4 <= 64 lanes, else 256-column passes; without a fused
    // epilogue (which needs the whole row in one group) passes are at most g_pass_cols wide.
    const int lanes = d / 4;
    int G = lanes >= 64 ? 64 : next_pow2(lanes);
    const int pass_cols = g_pass_cols ? g_pass_cols : (d <= 128 ? 256 : 64);
    if (!ex && 4 * G > pass_cols) G = pass_cols / 4;
    const int n_pass = (d + 4 * G - 1) / (4 * G);
    if (blk_seg) {  // source-blocked: every pass runs the blocks in order, the later ones adding
      // passes of up to 128 columns (unless tuned): at d = 256 the blocked hop into items takes
      // 16.99 ms in 128-column passes, 18.04 in 64-column ones and 19.54 in one 256-wide pass
      // (scripts/bench_mall_blocked.py --pass-cols, profiles/r06_round/wide/)
      const int bcols = g_pass_cols ? g_pass_cols : 128;
      G = lanes >= 64 ? 64 : next_pow2(lanes);
      if (4 * G > bcols) G = bcols / 4;
      for (int c0 = 0; c0 < d; c0 += 4 * G) {
        a.col0 = c0;
        for (int k = 0; k < n_blk; ++k) {
          a.rowptr = blk_seg + static_cast<int64_t>(k) * n_rows;  // block k's own CSR
          a.seg = g_blocked_seg;
          a.blk_accum = k > 0;
          a.epi = k + 1 == n_blk ? epilogue : HGD_EPI_NONE;  // the activation after the last
          hgd_status s = launch_vec<4>(G, a, has_val, st);
          if (s != HGD_OK) return s;
        }
      }
      return HGD_OK;
    }
    if (g_pass_interleave && n_pass > 1 && !ex && !mask && a.n_chunks == 0 && !a.seg) {
      a.col0 = 0;
      a.n_pass = n_pass;
      a.pass_cols = 4 * G;
      return launch_vec<4>(G, a, has_val, st);
    }
    for (int c0 = 0; c0 < d; c0 += 4 * G) {
      a.col0 = c0;
      hgd_status s = ex ? launch_vec<4, true>(G, a, has_val, st)
                        : launch_vec<4>(G, a, has_val, st);
      if (s != HGD_OK) return s;
    }
  } else {
    const int G = d >= 64 ? 64 : next_pow2(d);
    for (int c0 = 0; c0 < d; c0 += G) {
      a.col0 = c0;
      for (int k = 0; k < (blk_seg ? n_blk : 1); ++k) {
        if (blk_seg) {
          a.rowptr = blk_seg + static_cast<int64_t>(k) * n_rows;
          a.blk_accum = k > 0;
          a.epi = k + 1 == n_blk ? epilogue : HGD_EPI_NONE;
        }
        hgd_status s = ex ? launch_vec<1, true>(G, a, has_val, st)
                          : launch_vec<1>(G, a, has_val, st);
        if (s != HGD_OK) return s;
      }
    }
  }
  return HGD_OK;
}

// Source block of column c among n_blk ranges [⌊n_cols·k/n_blk⌋, ⌊n_cols·(k+1)/n_blk⌋), stepping
// k up from the previous nonzero's block (the columns of a row ascend).
__device__ __forceinline__ int32_t advance_block(int64_t c, int32_t k, int64_t n_cols,
                                                 int32_t n_blk) {
  while (k + 1 < n_blk && c >= n_cols * (k + 1) / n_blk) ++k;
  return k;
}

// cnt[k·n_rows + r] = nonzeros of row r in source block k (block-major, the order of the blocked
// copy); one thread per row walks it once. cnt[n_blk·n_rows] = 0 closes the scan.
__global__ void col_block_count_kernel(const int64_t* __restrict__ rowptr,
                                       const int32_t* __restrict__ col, int64_t n_rows,
                                       int64_t n_cols, int32_t n_blk, int64_t* __restrict__ cnt) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (r == 0) cnt[static_cast<int64_t>(n_blk) * n_rows] = 0;
  if (r >= n_rows) return;
  const int64_t b = rowptr[r], e = rowptr[r + 1];
  int32_t k = 0;
  int64_t start = b;
  for (int64_t i = b; i < e; ++i) {
    const int32_t kk = advance_block(col[i], k, n_cols, n_blk);
    if (kk != k) {
      cnt[static_cast<int64_t>(k) * n_rows + r] = i - start;
      for (int32_t j = k + 1; j < kk; ++j) cnt[static_cast<int64_t>(j) * n_rows + r] = 0;
      k = kk;
      start = i;
    }
  }
  cnt[static_cast<int64_t>(k) * n_rows + r] = e - start;
  for (int32_t j = k + 1; j < n_blk; ++j) cnt[static_cast<int64_t>(j) * n_rows + r] = 0;
}

// Moves every nonzero to its block-major position blk_start[k·n_rows + r] + (its rank inside the
// row's block k): blk_col gets the column, blk_perm (optional) the source position, with which
// any per-nonzero array of the structure is gathered into the same order.
__global__ void col_block_scatter_kernel(const int64_t* __restrict__ rowptr,
                                         const int32_t* __restrict__ col, int64_t n_rows,
                                         int64_t n_cols, int32_t n_blk,
                                         const int64_t* __restrict__ blk_start,
                                         int32_t* __restrict__ blk_col,
                                         int32_t* __restrict__ blk_perm) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (r >= n_rows) return;
  const int64_t b = rowptr[r], e = rowptr[r + 1];
  int32_t k = 0;
  int64_t start = b, out = blk_start[r];
  for (int64_t i = b; i < e; ++i) {
    const int32_t c = col[i];
    const int32_t kk = advance_block(c, k, n_cols, n_blk);
    if (kk != k) {
      k = kk;
      start = i;
      out = blk_start[static_cast<int64_t>(k) * n_rows + r];
    }
    blk_col[out + (i - start)] = c;
    if (blk_perm) blk_perm[out + (i - start)] = static_cast<int32_t>(i);
  }
}

}  // namespace
}  // namespace hgd

extern "C" hgd_status hgd_spmm(const int64_t* rowptr, const int32_t* col, const float* val,
                               const float* row_scale, int64_t n_rows, int64_t n_src_rows,
                               int64_t row_begin, int64_t row_end, const float* X, int64_t ldx,
                               float* Y, int64_t ldy, int32_t d, int32_t epilogue, float slope,
                               const hgd_split_plan* plan, void* workspace,
                               size_t workspace_bytes, void* stream) {
  hgd::clear_error();
  return hgd::spmm_impl(rowptr, col, val, row_scale, n_rows, n_src_rows, row_begin, row_end, X,
                        ldx, Y, ldy, d, epilogue, slope, nullptr, nullptr, 1.f, plan, workspace,
                        workspace_bytes, stream, "hgd_spmm");
}

extern "C" int32_t hgd_spmm_blocks_for(int64_t n_src_rows, int32_t d) {
  // one pass's gathered table: a blocked hop runs rows wider than 128 as 128-column passes
  const double table = static_cast<double>(n_src_rows) * (d < 128 ? d : 128) * 4.0;
  if (n_src_rows <= 0 || d <= 0 || table < 536870912.0) return 0;  // < 512 MiB: one pass
  if (table < 1073741824.0) return 2;                               // < 1 GiB: two blocks
  const double x = table / (640.0 * 1048576.0);                     // ~ one per 640 MiB
  double p = std::floor(x);  // rounded half to even
  const double frac = x - p;
  if (frac > 0.5 || (frac == 0.5 && std::fmod(p, 2.0) != 0.0)) p += 1.0;
  return static_cast<int32_t>(p < 4.0 ? 4.0 : (p > 16.0 ? 16.0 : p));
}

extern "C" size_t hgd_spmm_col_blocks_workspace_size(int64_t n_rows, int32_t n_blocks) {
  if (n_rows <= 0 || n_blocks <= 0) return 0;
  const int64_t n = static_cast<int64_t>(n_blocks) * n_rows + 1;
  size_t scan = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, scan, static_cast<const int64_t*>(nullptr),
                                       static_cast<int64_t*>(nullptr), n) != hipSuccess)
    return 0;
  return hgd::align_up(static_cast<size_t>(n) * sizeof(int64_t)) + hgd::align_up(scan);
}

extern "C" hgd_status hgd_spmm_col_blocks(const int64_t* rowptr, const int32_t* col,
                                          int64_t n_rows, int64_t n_cols, int32_t n_blocks,
                                          int64_t* blk_start, int32_t* blk_col,
                                          int32_t* blk_perm, void* workspace,
                                          size_t workspace_bytes, void* stream) {
  using namespace hgd;
  clear_error();
  HGD_REQUIRE(n_rows >= 0 && n_cols >= 0, "hgd_spmm_col_blocks: negative sizes");
  HGD_REQUIRE(n_blocks >= 1 && n_blocks <= 64, "hgd_spmm_col_blocks: blocks must be 1..64");
  HGD_REQUIRE(n_cols < (int64_t(1) << 31), "hgd_spmm_col_blocks: n_cols >= 2^31");
  if (n_rows == 0) return HGD_OK;
  HGD_REQUIRE(rowptr && blk_start, "hgd_spmm_col_blocks: null rowptr / blk_start");
  const size_t need = hgd_spmm_col_blocks_workspace_size(n_rows, n_blocks);
  if (!workspace || workspace_bytes < need)
    return fail(HGD_ERR_WORKSPACE, "hgd_spmm_col_blocks: workspace %zu < %zu", workspace_bytes,
                need);
  const int64_t grid = (n_rows + 255) / 256;
  HGD_REQUIRE(grid <= 0x7fffffffLL, "hgd_spmm_col_blocks: too many rows");
  hipStream_t st = as_stream(stream);
  const int64_t n = static_cast<int64_t>(n_blocks) * n_rows + 1;
  int64_t* cnt = static_cast<int64_t*>(workspace);
  char* tmp = static_cast<char*>(workspace) + align_up(static_cast<size_t>(n) * sizeof(int64_t));
  size_t tmp_bytes = workspace_bytes - align_up(static_cast<size_t>(n) * sizeof(int64_t));
  hipLaunchKernelGGL(col_block_count_kernel, dim3(grid), dim3(256), 0, st, rowptr, col, n_rows,
                     n_cols, n_blocks, cnt);
  hgd_status s = check_launch("hgd_spmm_col_blocks count");
  if (s != HGD_OK) return s;
  HGD_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, cnt, blk_start, n, st));
  hipLaunchKernelGGL(col_block_scatter_kernel, dim3(grid), dim3(256), 0, st, rowptr, col, n_rows,
                     n_cols, n_blocks, blk_start, blk_col, blk_perm);
  return check_launch("hgd_spmm_col_blocks scatter");
}

extern "C" hgd_status hgd_spmm_blocked(const int64_t* blk_start, const int32_t* blk_col,
                                       const float* blk_val, const float* row_scale,
                                       int64_t n_rows, int64_t n_src_rows, int64_t row_begin,
                                       int64_t row_end, const float* X, int64_t ldx, float* Y,
                                       int64_t ldy, int32_t d, int32_t epilogue, float slope,
                                       int32_t n_blocks, void* stream) {
  hgd::clear_error();
  HGD_REQUIRE(n_blocks >= 1 && n_blocks <= 64, "hgd_spmm_blocked: blocks must be 1..64");
  HGD_REQUIRE(row_end <= row_begin || blk_start, "hgd_spmm_blocked: null blk_start");
  // spmm_impl's rowptr argument is only checked for NULL on this path
  return hgd::spmm_impl(blk_start, blk_col, blk_val, row_scale, n_rows, n_src_rows, row_begin,
                        row_end, X, ldx, Y, ldy, d, epilogue, slope, nullptr, nullptr, 1.f,
                        nullptr, nullptr, 0, stream, "hgd_spmm_blocked", blk_start, n_blocks);
}

extern "C" hgd_status hgd_spmm_fused(const int64_t* rowptr, const int32_t* col, const float* val,
                                     const float* row_scale, int64_t n_rows, int64_t n_src_rows,
                                     int64_t row_begin, int64_t row_end, const float* X,
                                     int64_t ldx, float* Y, int64_t ldy, int32_t d,
                                     const hgd_row_epilogue* epi, const hgd_split_plan* plan,
                                     void* workspace, size_t workspace_bytes, void* stream) {
  hgd::clear_error();
  HGD_REQUIRE(epi != nullptr, "hgd_spmm_fused: null epilogue descriptor");
  return hgd::spmm_impl(rowptr, col, val, row_scale, n_rows, n_src_rows, row_begin, row_end, X,
                        ldx, Y, ldy, d, epi->act, epi->slope, epi, nullptr, 1.f, plan, workspace,
                        workspace_bytes, stream, "hgd_spmm_fused");
}

extern "C" hgd_status hgd_spmm_masked(const int64_t* rowptr, const int32_t* col, const float* val,
                                      const uint8_t* mask, float keep, const float* row_scale,
                                      int64_t n_rows, int64_t n_src_rows, int64_t row_begin,
                                      int64_t row_end, const float* X, int64_t ldx, float* Y,
                                      int64_t ldy, int32_t d, int32_t epilogue, float slope,
                                      const hgd_split_plan* plan, void* workspace,
                                      size_t workspace_bytes, void* stream) {
  hgd::clear_error();
  HGD_REQUIRE(keep > 0.f, "hgd_spmm_masked: keep must be > 0 (got %g)", (double)keep);
  HGD_REQUIRE(mask || row_end == row_begin, "hgd_spmm_masked: null mask");
  return hgd::spmm_impl(rowptr, col, val, row_scale, n_rows, n_src_rows, row_begin, row_end, X,
                        ldx, Y, ldy, d, epilogue, slope, nullptr, mask, keep, plan, workspace,
                        workspace_bytes, stream, "hgd_spmm_masked");
}

extern "C" hgd_status hgd_spmm_masked_fused(const int64_t* rowptr, const int32_t* col,
                                            const float* val, const uint8_t* mask, float keep,
                                            const float* row_scale, int64_t n_rows,
                                            int64_t n_src_rows, int64_t row_begin,
                                            int64_t row_end, const float* X, int64_t ldx,
                                            float* Y, int64_t ldy, int32_t d,
                                            const hgd_row_epilogue* epi,
                                            const hgd_split_plan* plan, void* workspace,
                                            size_t workspace_bytes, void* stream) {
  hgd::clear_error();
  HGD_REQUIRE(epi != nullptr, "hgd_spmm_masked_fused: null epilogue descriptor");
  HGD_REQUIRE(keep > 0.f, "hgd_spmm_masked_fused: keep must be > 0 (got %g)", (double)keep);
  HGD_REQUIRE(mask || row_end == row_begin, "hgd_spmm_masked_fused: null mask");
  return hgd::spmm_impl(rowptr, col, val, row_scale, n_rows, n_src_rows, row_begin, row_end, X,
                        ldx, Y, ldy, d, epi->act, epi->slope, epi, mask, keep, plan, workspace,
                        workspace_bytes, stream, "hgd_spmm_masked_fused");
}

extern "C" hgd_status hgd_set_tuning(int32_t key, int32_t value) {
  using namespace hgd;
  clear_error();
  switch (key) {
    case HGD_TUNE_SPMM_UNROLL:
      HGD_REQUIRE(value == 8 || value == 16, "hgd_set_tuning: unroll must be 8 or 16");
      g_unroll = value;
      return HGD_OK;
    case HGD_TUNE_SPMM_POLICY:
      HGD_REQUIRE(value == 0 || value == 1 || (value >= 8 && value <= 11),
                  "hgd_set_tuning: policy must be 0, 1 (nt stores), 8 (index prefetch), 9, 10 "
                  "(prefetch + nt index loads) or 11");
      g_policy = value;
      return HGD_OK;
    case HGD_TUNE_SPMM_PASS_COLS:
      HGD_REQUIRE(value == 0 || value == 64 || value == 128 || value == 256,
                  "hgd_set_tuning: pass columns must be 0 (auto), 64, 128 or 256");
      g_pass_cols = value;
      return HGD_OK;
    case HGD_TUNE_ROWGEMM_BLOCKS:
      HGD_REQUIRE(value == 0 || (value >= 64 && value <= 8192),
                  "hgd_set_tuning: row-GEMM blocks must be 0 (default) or in [64, 8192]");
      set_row_gemm_max_blocks(value);
      return HGD_OK;
    case HGD_TUNE_SPLITK_ROWS:
      HGD_REQUIRE(value == 0 || (value >= 64 && value <= 65536 && value % 64 == 0),
                  "hgd_set_tuning: split-K rows must be 0 (default) or a multiple of 64 in "
                  "[64, 65536]");
      set_splitk_rows(value);
      return HGD_OK;
    case HGD_TUNE_GEMM_EXACT:
      HGD_REQUIRE(value == 0 || value == 1, "hgd_set_tuning: gemm exact must be 0 or 1");
      set_gemm_exact(value);
      return HGD_OK;
    case HGD_TUNE_X3_COLS:
      HGD_REQUIRE(value == 0 || value == 64 || value == 128,
                  "hgd_set_tuning: x3 columns must be 0 (default), 64 or 128");
      set_x3_cols(value);
      return HGD_OK;
    case HGD_TUNE_X3_SPLITK:
      HGD_REQUIRE(value >= 0 && value <= 2, "hgd_set_tuning: x3 split-K must be 0, 1 or 2");
      set_x3_splitk(value);
      return HGD_OK;
    case HGD_TUNE_X3S_TILES:
      HGD_REQUIRE(value >= 0 && value <= 3, "hgd_set_tuning: x3s tiles must be 0, 1, 2 or 3");
      set_x3s_tiles(value);
      return HGD_OK;
    case HGD_TUNE_P2P_SEGMENT_MB:
      HGD_REQUIRE(value >= 0 && value <= 65536,
                  "hgd_set_tuning: p2p segment must be 0 (default) or 1..65536 MiB");
      set_p2p_segment_mb(value);
      return HGD_OK;
    case HGD_TUNE_P2P_CACHED:
      HGD_REQUIRE(value == 0 || value == 1, "hgd_set_tuning: p2p cached must be 0 or 1");
      set_p2p_cached(value);
      return HGD_OK;
    case HGD_TUNE_X3P_QUEUE:
      HGD_REQUIRE(value == 0 || value == 1, "hgd_set_tuning: x3p queue must be 0 or 1");
      set_x3p_queue(value);
      return HGD_OK;
    case HGD_TUNE_P2P_GRID:
      HGD_REQUIRE(value >= 0 && value <= 65536, "hgd_set_tuning: p2p grid must be 0..65536");
      set_p2p_grid(value);
      return HGD_OK;
    case HGD_TUNE_MASK_PAIR:
      HGD_REQUIRE(value >= 0 && value <= 2, "hgd_set_tuning: mask pair must be 0, 1 or 2");
      g_mask_pair = value;
      return HGD_OK;
    case HGD_TUNE_MASK_DIV:
      HGD_REQUIRE(value == 0 || value == 1, "hgd_set_tuning: mask div must be 0 or 1");
      g_mask_div = value;
      return HGD_OK;
    case HGD_TUNE_SPMM_PASS_INTERLEAVE:
      HGD_REQUIRE(value == 0 || value == 1, "hgd_set_tuning: pass interleave must be 0 or 1");
      g_pass_interleave = value;
      return HGD_OK;
    case HGD_TUNE_SPMM_BLOCKED_SEG:
      HGD_REQUIRE(value == 0 || value == 1, "hgd_set_tuning: blocked seg must be 0 or 1");
      g_blocked_seg = value;
      return HGD_OK;
    case HGD_TUNE_CPU_RNG_THREADS:
      HGD_REQUIRE(value >= 0 && value <= 64, "hgd_set_tuning: cpu rng threads must be 0..64");
      set_cpu_rng_threads(value);
      return HGD_OK;
    default:
      return fail(HGD_ERR_INVALID_ARG, "hgd_set_tuning: unknown key %d", key);
  }
}
