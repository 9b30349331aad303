// Backward of the fused row epilogue of hgd_spmm_fused (include/hgd.h, hgd_row_epilogue).
//
// The forward (spmm.hip, finish_row) computed, per row, a = act(z), b = LN(a)·γ + β and
// Y = out_scale·b + residuals. Here, with the same one-lane-group-per-row mapping (G = d/4 lanes
// × float4 at d = 64), dZ = act'(a) ⊙ LN_bwd(out_scale·dY) in one pass over dY and act_out — the
// reference runs LayerNorm backward, the add / blend backward and the LeakyReLU backward as
// separate torch kernels, each an [N, d] round trip (model/layers/EquivSetConv.py:86-107).
// dγ / dβ are column sums over all rows: every block folds its rows into per-lane registers,
// combines its lane groups in LDS in group order and writes one partial row; a second kernel sums
// the partials in block order. The grid size depends only on (n_rows, d), so the result is
// deterministic run to run.
#include "device_util.h"
#include "hgd_internal.h"

namespace hgd {
namespace {

constexpr int kMaxBlocks = 1024;

struct RowEpiBwd {
  const float* dY;
  int64_t ldy;
  const float* A;
  int64_t lda;
  const float* stats;
  const float* gamma;
  int64_t n;
  int32_t d;
  int32_t col0;
  int32_t act;
  float slope;
  int32_t ln;
  float out_scale;
  float* dZ;
  int64_t ldz;
  float* part_g;  // [gridDim.x, d] or NULL
  float* part_b;
};

template <int G, int VEC>
__global__ __launch_bounds__(kBlock) void k_rowepi_bwd(RowEpiBwd p) {
  constexpr int GPB = kBlock / G;
  __shared__ float s_g[GPB * G * VEC];
  __shared__ float s_b[GPB * G * VEC];
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  const int64_t coff = static_cast<int64_t>(p.col0) + static_cast<int64_t>(l) * VEC;
  const bool col_ok = coff < p.d;
  const bool need_a = p.ln || p.act != HGD_EPI_NONE;
  float gm[VEC], acc_g[VEC], acc_b[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    gm[i] = (p.gamma && col_ok) ? p.gamma[coff + i] : 1.f;
    acc_g[i] = 0.f;
    acc_b[i] = 0.f;
  }
  const float inv_d = 1.f / static_cast<float>(p.d);
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * GPB + g; r < p.n;
       r += static_cast<int64_t>(gridDim.x) * GPB) {
    float dy[VEC], a[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) dy[i] = a[i] = 0.f;
    if (col_ok) {
      load_vec<VEC>(p.dY + r * p.ldy + coff, dy);
      if (need_a) load_vec<VEC>(p.A + r * p.lda + coff, a);
    }
#pragma unroll
    for (int i = 0; i < VEC; ++i) dy[i] *= p.out_scale;
    float da[VEC];
    if (p.ln) {
      const float mu = p.stats[2 * r];
      const float rstd = p.stats[2 * r + 1];
      float ah[VEC], gh[VEC];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        ah[i] = (a[i] - mu) * rstd;
        gh[i] = dy[i] * gm[i];
        if (col_ok) {
          s1 += gh[i];
          s2 += gh[i] * ah[i];
          acc_g[i] = fmaf(dy[i], ah[i], acc_g[i]);
          acc_b[i] += dy[i];
        }
      }
      s1 = group_sum<G>(s1) * inv_d;
      s2 = group_sum<G>(s2) * inv_d;
#pragma unroll
      for (int i = 0; i < VEC; ++i) da[i] = rstd * (gh[i] - s1 - ah[i] * s2);
    } else {
#pragma unroll
      for (int i = 0; i < VEC; ++i) da[i] = dy[i];
    }
    if (p.act == HGD_EPI_LEAKY_RELU) {
#pragma unroll
      for (int i = 0; i < VEC; ++i) da[i] = a[i] > 0.f ? da[i] : da[i] * p.slope;
    } else if (p.act == HGD_EPI_RELU) {
#pragma unroll
      for (int i = 0; i < VEC; ++i) da[i] = a[i] > 0.f ? da[i] : 0.f;
    }
    if (col_ok) store_vec<VEC>(p.dZ + r * p.ldz + coff, da);
  }
  if (!p.part_g) return;  // block-uniform
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    s_g[g * G * VEC + l * VEC + i] = acc_g[i];
    s_b[g * G * VEC + l * VEC + i] = acc_b[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < p.d; c += kBlock) {
    float sg = 0.f, sb = 0.f;
    for (int k = 0; k < GPB; ++k) {
      sg += s_g[k * G * VEC + c];
      sb += s_b[k * G * VEC + c];
    }
    p.part_g[static_cast<int64_t>(blockIdx.x) * p.d + c] = sg;
    p.part_b[static_cast<int64_t>(blockIdx.x) * p.d + c] = sb;
  }
}

// Forward of the row epilogue on an existing matrix Z (hgd_row_epilogue_forward): the same math
// as hgd_spmm_fused's store, for the LayerNorms that do not follow a hop (the MLP InputNorm of
// model/layers/MLP.py:65-71,109-110). One lane group per row; statistics by group_sum.
struct RowEpiFwd {
  const float* Z;
  int64_t ldz;
  int64_t n;
  int32_t d;
  hgd_row_epilogue e;
  float* Y;
  int64_t ldy;
};

template <int G, int VEC>
__global__ __launch_bounds__(kBlock) void k_rowepi_fwd(RowEpiFwd p) {
  constexpr int GPB = kBlock / G;
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  const int64_t coff = static_cast<int64_t>(l) * VEC;
  const bool col_ok = coff < p.d;
  const hgd_row_epilogue& e = p.e;
  const float inv_d = 1.f / static_cast<float>(p.d);
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * GPB + g; r < p.n;
       r += static_cast<int64_t>(gridDim.x) * GPB) {
    float v[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) v[i] = 0.f;
    if (col_ok) load_vec<VEC>(p.Z + r * p.ldz + coff, v);
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      if (e.act == HGD_EPI_LEAKY_RELU) v[i] = v[i] > 0.f ? v[i] : v[i] * e.slope;
      else if (e.act == HGD_EPI_RELU) v[i] = v[i] > 0.f ? v[i] : 0.f;
    }
    if (e.act_out && col_ok) store_vec<VEC>(e.act_out + r * e.ld_act + coff, v);
    if (e.layer_norm) {
      float t = 0.f;
      if (col_ok) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) t += v[i];
      }
      const float mu = group_sum<G>(t) * inv_d;
      t = 0.f;
      if (col_ok) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) t += (v[i] - mu) * (v[i] - mu);
      }
      const float rstd = 1.f / sqrtf(group_sum<G>(t) * inv_d + e.ln_eps);
      if (e.stats && l == 0) {
        e.stats[2 * r] = mu;
        e.stats[2 * r + 1] = rstd;
      }
      if (col_ok) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const float gm = e.ln_gamma ? e.ln_gamma[coff + i] : 1.f;
          const float bt = e.ln_beta ? e.ln_beta[coff + i] : 0.f;
          v[i] = fmaf((v[i] - mu) * rstd, gm, bt);
        }
      }
    }
    if (!col_ok) continue;
#pragma unroll
    for (int i = 0; i < VEC; ++i) v[i] *= e.out_scale;
    if (e.res1) {
      float rv[VEC];
      load_vec<VEC>(e.res1 + r * e.ld_res1 + coff, rv);
#pragma unroll
      for (int i = 0; i < VEC; ++i) v[i] = fmaf(e.res1_scale, rv[i], v[i]);
    }
    if (e.res2) {
      float rv[VEC];
      load_vec<VEC>(e.res2 + r * e.ld_res2 + coff, rv);
#pragma unroll
      for (int i = 0; i < VEC; ++i) v[i] = fmaf(e.res2_scale, rv[i], v[i]);
    }
    store_vec<VEC>(p.Y + r * p.ldy + coff, v);
    if (e.sum_out) {
      float rv[VEC];
      load_vec<VEC>(e.sum_res + r * e.ld_sum_res + coff, rv);
#pragma unroll
      for (int i = 0; i < VEC; ++i) rv[i] += v[i];
      store_vec<VEC>(e.sum_out + r * e.ld_sum_out + coff, rv);
    }
  }
}

template <int VEC>
hgd_status launch(int G, const RowEpiBwd& p, int64_t blocks, hipStream_t st) {
  switch (G) {
#define HGD_CASE(GG)                                                                      \
    case GG:                                                                              \
      hipLaunchKernelGGL((k_rowepi_bwd<GG, VEC>), dim3(blocks), dim3(kBlock), 0, st, p);  \
      return check_launch("hgd_row_epilogue_backward");
    HGD_CASE(1) HGD_CASE(2) HGD_CASE(4) HGD_CASE(8) HGD_CASE(16) HGD_CASE(32) HGD_CASE(64)
#undef HGD_CASE
    default:
      return fail(HGD_ERR_UNSUPPORTED, "hgd_row_epilogue_backward: group size %d", G);
  }
}

template <int VEC>
hgd_status launch_fwd(int G, const RowEpiFwd& p, int64_t blocks, hipStream_t st) {
  switch (G) {
#define HGD_CASE(GG)                                                                      \
    case GG:                                                                              \
      hipLaunchKernelGGL((k_rowepi_fwd<GG, VEC>), dim3(blocks), dim3(kBlock), 0, st, p);  \
      return check_launch("hgd_row_epilogue_forward");
    HGD_CASE(1) HGD_CASE(2) HGD_CASE(4) HGD_CASE(8) HGD_CASE(16) HGD_CASE(32) HGD_CASE(64)
#undef HGD_CASE
    default:
      return fail(HGD_ERR_UNSUPPORTED, "hgd_row_epilogue_forward: group size %d", G);
  }
}

int64_t grid_blocks(int64_t n_rows, int G) {
  const int64_t gpb = kBlock / G;
  int64_t b = (n_rows + gpb - 1) / gpb;
  if (b > kMaxBlocks) b = kMaxBlocks;
  return b < 1 ? 1 : b;
}

}  // namespace
}  // namespace hgd

extern "C" size_t hgd_row_epilogue_backward_workspace_size(int64_t n_rows, int32_t d) {
  if (n_rows <= 0 || d <= 0) return 0;
  return 2 * hgd::align_up(static_cast<size_t>(hgd::kMaxBlocks) * static_cast<size_t>(d) * 4);
}

extern "C" hgd_status hgd_row_epilogue_backward(const float* dY, int64_t ldy, const float* act_out,
                                                int64_t ld_act, const float* stats,
                                                const float* ln_gamma, int64_t n_rows, int32_t d,
                                                int32_t act, float slope, int32_t layer_norm,
                                                float out_scale, float* dZ, int64_t ldz,
                                                float* dgamma, float* dbeta, void* workspace,
                                                size_t workspace_bytes, void* stream) {
  using namespace hgd;
  clear_error();
  HGD_REQUIRE(d > 0 && n_rows >= 0, "hgd_row_epilogue_backward: bad sizes");
  HGD_REQUIRE(act >= HGD_EPI_NONE && act <= HGD_EPI_RELU, "hgd_row_epilogue_backward: bad act");
  HGD_REQUIRE(act == HGD_EPI_NONE || slope >= 0.f,
              "hgd_row_epilogue_backward: activation needs slope >= 0");
  HGD_REQUIRE(layer_norm == 0 || layer_norm == 1, "hgd_row_epilogue_backward: layer_norm 0/1");
  HGD_REQUIRE(ldy >= d && ldz >= d, "hgd_row_epilogue_backward: ldy/ldz < d");
  const bool need_a = layer_norm || act != HGD_EPI_NONE;
  if (n_rows == 0) {
    if (layer_norm && (dgamma || dbeta)) {
      hipStream_t st = as_stream(stream);
      if (dgamma) HGD_HIP(hipMemsetAsync(dgamma, 0, static_cast<size_t>(d) * 4, st));
      if (dbeta) HGD_HIP(hipMemsetAsync(dbeta, 0, static_cast<size_t>(d) * 4, st));
    }
    return HGD_OK;
  }
  HGD_REQUIRE(dY && dZ, "hgd_row_epilogue_backward: null dY/dZ");
  HGD_REQUIRE(!need_a || (act_out && ld_act >= d), "hgd_row_epilogue_backward: act_out required");
  HGD_REQUIRE(!layer_norm || stats, "hgd_row_epilogue_backward: stats required for layer_norm");
  auto al16 = [](const void* p, int64_t ld) {
    return p == nullptr || (reinterpret_cast<uintptr_t>(p) % 16 == 0 && ld % 4 == 0);
  };
  const bool aligned =
      d % 4 == 0 && al16(dY, ldy) && al16(dZ, ldz) && al16(need_a ? act_out : nullptr, ld_act);
  const int G = aligned ? (d / 4 >= 64 ? 64 : next_pow2(d / 4)) : (d >= 64 ? 64 : next_pow2(d));
  const int span = aligned ? 4 * G : G;
  if (layer_norm && span < d)
    return fail(HGD_ERR_UNSUPPORTED,
                "hgd_row_epilogue_backward: layer_norm needs d <= 256 (aligned) or <= 64");
  const bool want_gb = layer_norm && (dgamma || dbeta);
  const int64_t blocks = grid_blocks(n_rows, G);
  if (want_gb) {
    const size_t need = hgd_row_epilogue_backward_workspace_size(n_rows, d);
    if (workspace_bytes < need || !workspace)
      return fail(HGD_ERR_WORKSPACE, "hgd_row_epilogue_backward: workspace %zu < required %zu",
                  workspace_bytes, need);
  }
  RowEpiBwd p{};
  p.dY = dY;
  p.ldy = ldy;
  p.A = act_out;
  p.lda = ld_act;
  p.stats = stats;
  p.gamma = ln_gamma;
  p.n = n_rows;
  p.d = d;
  p.act = act;
  p.slope = slope;
  p.ln = layer_norm;
  p.out_scale = out_scale;
  p.dZ = dZ;
  p.ldz = ldz;
  if (want_gb) {
    p.part_g = static_cast<float*>(workspace);
    p.part_b = reinterpret_cast<float*>(static_cast<char*>(workspace) +
                                        align_up(static_cast<size_t>(kMaxBlocks) * d * 4));
  }
  hipStream_t st = as_stream(stream);
  for (int c0 = 0; c0 < d; c0 += span) {
    p.col0 = c0;
    hgd_status s = aligned ? launch<4>(G, p, blocks, st) : launch<1>(G, p, blocks, st);
    if (s != HGD_OK) return s;
  }
  if (want_gb) {
    if (dgamma) {
      hgd_status s = sum_rows(p.part_g, blocks, d, dgamma, st);
      if (s != HGD_OK) return s;
    }
    if (dbeta) return sum_rows(p.part_b, blocks, d, dbeta, st);
  }
  return HGD_OK;
}

extern "C" hgd_status hgd_row_epilogue_forward(const float* Z, int64_t ldz, int64_t n_rows,
                                               int32_t d, const hgd_row_epilogue* epi, float* Y,
                                               int64_t ldy, void* stream) {
  using namespace hgd;
  clear_error();
  HGD_REQUIRE(epi != nullptr, "hgd_row_epilogue_forward: null epilogue descriptor");
  HGD_REQUIRE(d > 0 && n_rows >= 0, "hgd_row_epilogue_forward: bad sizes");
  HGD_REQUIRE(epi->act >= HGD_EPI_NONE && epi->act <= HGD_EPI_RELU,
              "hgd_row_epilogue_forward: bad act");
  HGD_REQUIRE(epi->act == HGD_EPI_NONE || epi->slope >= 0.f,
              "hgd_row_epilogue_forward: activation needs slope >= 0");
  HGD_REQUIRE(epi->layer_norm == 0 || epi->layer_norm == 1,
              "hgd_row_epilogue_forward: layer_norm 0/1");
  HGD_REQUIRE(ldz >= d && ldy >= d, "hgd_row_epilogue_forward: ldz/ldy < d");
  HGD_REQUIRE((!epi->res1 || epi->ld_res1 >= d) && (!epi->res2 || epi->ld_res2 >= d) &&
                  (!epi->act_out || epi->ld_act >= d) &&
                  (!epi->sum_out || (epi->ld_sum_out >= d && epi->ld_sum_res >= d)),
              "hgd_row_epilogue_forward: leading dimension < d");
  HGD_REQUIRE((epi->sum_out == nullptr) == (epi->sum_res == nullptr),
              "hgd_row_epilogue_forward: sum_out and sum_res go together");
  if (n_rows == 0) return HGD_OK;
  HGD_REQUIRE(Z && Y, "hgd_row_epilogue_forward: null Z/Y");
  auto al16 = [](const void* p, int64_t ld) {
    return p == nullptr || (reinterpret_cast<uintptr_t>(p) % 16 == 0 && ld % 4 == 0);
  };
  const bool aligned = d % 4 == 0 && al16(Z, ldz) && al16(Y, ldy) &&
                       al16(epi->res1, epi->ld_res1) && al16(epi->res2, epi->ld_res2) &&
                       al16(epi->act_out, epi->ld_act) && al16(epi->sum_out, epi->ld_sum_out) &&
                       al16(epi->sum_res, epi->ld_sum_res);
  const int G = aligned ? (d / 4 >= 64 ? 64 : next_pow2(d / 4)) : (d >= 64 ? 64 : next_pow2(d));
  const int span = aligned ? 4 * G : G;
  if (span < d)
    return fail(HGD_ERR_UNSUPPORTED,
                "hgd_row_epilogue_forward: needs d <= 256 (aligned rows) or d <= 64 (got %d)", d);
  RowEpiFwd p{};
  p.Z = Z;
  p.ldz = ldz;
  p.n = n_rows;
  p.d = d;
  p.e = *epi;
  p.Y = Y;
  p.ldy = ldy;
  const int64_t gpb = kBlock / G;
  int64_t blocks = (n_rows + gpb - 1) / gpb;
  if (blocks > 4096) blocks = 4096;
  return aligned ? launch_fwd<4>(G, p, blocks, as_stream(stream))
                 : launch_fwd<1>(G, p, blocks, as_stream(stream));
}
