// BPR loss of a recommender batch straight from the embedding table (util/loss_torch.py:5-9 on
// the rows model/graph/HCCF.py:84-86 gathers):
//   anc = E[uid], pos = E[nu + pid], neg = E[nu + nid]
//   loss = mean_k −log(1e-5 + σ(⟨anc_k, pos_k⟩ − ⟨anc_k, neg_k⟩))
// In the reference these are three index gathers, two mul + sum pairs, sub, sigmoid, add, log,
// neg and mean forward, and the same chain backward ending in three sort-based index_put
// scatters (~40 small launches per step). Here: forward = one row kernel (gather, both dots,
// per-row term and backward coefficient) + one fixed-order reduction; backward = zero/init,
// one pass linking every position into its destination row's list (integer atomics), and one
// row kernel in which one position per destination sums the contributions of all the row's
// positions in ascending position order — deterministic, no float atomics, no sort.
#include <algorithm>

#include "device_util.h"
#include "hgd_internal.h"

namespace hgd {
namespace {

struct BprArgs {
  const float* E;
  int64_t lde;
  int64_t nu, ni;
  const int64_t* uid;
  const int64_t* pid;
  const int64_t* nid;
  int64_t B;
  int32_t d;
};

// torch indexing semantics for a valid index (negatives wrap); out-of-range ids are clamped so
// a bad batch can never fault — the forward counts them into the caller's bad_index word (the
// reference's E[idx] gather raises; the host checks the count, functional.bpr_index_errors)
__device__ __forceinline__ bool index_ok(int64_t i, int64_t n) { return i >= -n && i < n; }

__device__ __forceinline__ int64_t fix_index(int64_t i, int64_t n) {
  if (i < 0) i += n;
  return i < 0 ? 0 : (i >= n ? n - 1 : i);
}

// table row of position q in [0, 3B): anchors, then positives, then negatives
__device__ __forceinline__ int64_t dest_row(const BprArgs& a, int64_t q) {
  if (q < a.B) return fix_index(a.uid[q], a.nu);
  if (q < 2 * a.B) return a.nu + fix_index(a.pid[q - a.B], a.ni);
  return a.nu + fix_index(a.nid[q - 2 * a.B], a.ni);
}

template <int G>
__global__ __launch_bounds__(kBlock) void k_bpr_rows(BprArgs a, float* anc_out, float* pos_out,
                                                    float* term, float* coef, int* bad) {
  constexpr int GPB = kBlock / G;
  const int l = threadIdx.x % G;
  const int64_t k = static_cast<int64_t>(blockIdx.x) * GPB + threadIdx.x / G;
  if (k >= a.B) return;
  const int64_t ru = dest_row(a, k), rp = dest_row(a, a.B + k), rn = dest_row(a, 2 * a.B + k);
  float sp = 0.f, sn = 0.f;
  for (int c = 4 * l; c < a.d; c += 4 * G) {
    float u[4], p[4], n[4];
    load_vec<4>(a.E + ru * a.lde + c, u);
    load_vec<4>(a.E + rp * a.lde + c, p);
    load_vec<4>(a.E + rn * a.lde + c, n);
    if (anc_out) store_vec<4>(anc_out + k * a.d + c, u);
    if (pos_out) store_vec<4>(pos_out + k * a.d + c, p);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      sp = fmaf(u[i], p[i], sp);
      sn = fmaf(u[i], n[i], sn);
    }
  }
  sp = group_sum<G>(sp);
  sn = group_sum<G>(sn);
  if (l == 0) {
    if (bad && !(index_ok(a.uid[k], a.nu) && index_ok(a.pid[k], a.ni) && index_ok(a.nid[k], a.ni)))
      atomicAdd(bad, 1);
    const float s = sp - sn;
    const float sig = 1.f / (1.f + expf(-s));
    const float den = 1e-5f + sig;
    term[k] = -logf(den);
    coef[k] = sig * (1.f - sig) / den;  // d(−log(1e-5 + σ(s)))/ds = −coef
  }
}

// loss = Σ term / B in a fixed order (one workgroup)
__global__ __launch_bounds__(1024) void k_bpr_mean(const float* term, int64_t B, float* loss) {
  __shared__ float s[1024];
  float acc = 0.f;
  for (int64_t i = threadIdx.x; i < B; i += 1024) acc += term[i];
  s[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if (static_cast<int>(threadIdx.x) < w) s[threadIdx.x] += s[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = s[0] / static_cast<float>(B);
}

__global__ void k_bpr_bwd_init(float* dE, int64_t lde, int64_t n_rows, int32_t d, int* head) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t per = d / 4;
  if (i < n_rows * per) {
    const int64_t r = i / per, c = 4 * (i % per);
    const float z[4] = {0.f, 0.f, 0.f, 0.f};
    store_vec<4>(dE + r * lde + c, z);
  }
  if (i < n_rows) head[i] = -1;
}

// Every position pushes itself onto its destination row's list (integer atomics; the list
// ORDER depends on timing, the set does not — the row kernel sorts it).
__global__ void k_bpr_bwd_link(BprArgs a, int* head, int* next, int* dst) {
  const int64_t q = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (q >= 3 * a.B) return;
  const int r = static_cast<int>(dest_row(a, q));
  dst[q] = r;
  next[q] = atomicExch(head + r, static_cast<int>(q));
}

// One lane group per position; the position left at the head of each destination row's list
// writes that row: the contributions of all its positions, summed in ascending position order.
// The list is walked ONCE into the group's LDS slots (up to CAP positions), ranked there (each
// lane counts the smaller entries of its slots) and added in rank order. Repeats are routine in
// real batches — a popular item is the positive of tens of batch rows, and at d = 32 a group is
// 4 lanes — so the ranking must not chase the list per element. A list longer than CAP (a
// skewed catalogue's head item: under Zipf(1.2) popularity one item is the positive of ~740 of
// 4,096 rows) stops being walked at CAP + 1 — a dependent load per entry — and the group scans
// the destination array instead, K positions per lane per step (independent loads), taking its
// row's positions in ascending order from the lanes' hit masks. That scan is ≤ 3B/(K·G) steps
// for the few such rows; the round-3 fallback (repeated minimum walks over the list, quadratic
// in dependent loads) took 45 ms per call on that batch.
template <int G>
__global__ __launch_bounds__(kBlock) void k_bpr_bwd_rows(BprArgs a, const float* coef,
                                                        const float* grad, const int* head,
                                                        const int* next, const int* dst,
                                                        float* dE, int64_t ldd) {
  constexpr int GPB = kBlock / G;
  const int l = threadIdx.x % G;
  const int64_t q = static_cast<int64_t>(blockIdx.x) * GPB + threadIdx.x / G;
  if (q >= 3 * a.B) return;
  constexpr int CAP = G >= 4 ? 64 : 16;
  __shared__ int s_list[GPB][CAP];
  __shared__ int s_sorted[GPB][CAP];
  const int grp = threadIdx.x / G;
  const int r = dst[q];
  if (head[r] != static_cast<int>(q)) return;  // group-uniform
  const float gB = -(*grad) / static_cast<float>(a.B);
  constexpr int NV = 4;  // float4 column blocks per lane: d / 4 <= NV·G for every group_for(d)
  float acc[NV][4];
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[v][i] = 0.f;
  auto add = [&](int64_t j) {
    const int64_t k = j < a.B ? j : (j < 2 * a.B ? j - a.B : j - 2 * a.B);
    const float t = gB * coef[k];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = 4 * (l + v * G);
      if (c >= a.d) break;
      if (j < a.B) {  // anchor: t·(pos − neg)
        float p[4], n[4];
        load_vec<4>(a.E + static_cast<int64_t>(dst[a.B + k]) * a.lde + c, p);
        load_vec<4>(a.E + static_cast<int64_t>(dst[2 * a.B + k]) * a.lde + c, n);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[v][i] += t * (p[i] - n[i]);
      } else {  // positive: t·anc, negative: −t·anc
        float u[4];
        load_vec<4>(a.E + static_cast<int64_t>(dst[k]) * a.lde + c, u);
        const float s = j < 2 * a.B ? t : -t;
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[v][i] += s * u[i];
      }
    }
  };
  // add(js[0]) … add(js[cnt-1]) in that order, the rows of all of them loaded first
  auto add4 = [&](const int64_t (&js)[4], int cnt) {
    float t4[4];
    int64_t k4[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j = js[u];
      k4[u] = j < a.B ? j : (j < 2 * a.B ? j - a.B : j - 2 * a.B);
      t4[u] = u < cnt ? gB * coef[k4[u]] : 0.f;
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = 4 * (l + v * G);
      if (c >= a.d) break;
      float r1[4][4], r2[4][4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u >= cnt) continue;
        if (js[u] < a.B) {
          load_vec<4>(a.E + static_cast<int64_t>(dst[a.B + k4[u]]) * a.lde + c, r1[u]);
          load_vec<4>(a.E + static_cast<int64_t>(dst[2 * a.B + k4[u]]) * a.lde + c, r2[u]);
        } else {
          load_vec<4>(a.E + static_cast<int64_t>(dst[k4[u]]) * a.lde + c, r1[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u >= cnt) continue;
        if (js[u] < a.B) {
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[v][i] += t4[u] * (r1[u][i] - r2[u][i]);
        } else {
          const float sg = js[u] < 2 * a.B ? t4[u] : -t4[u];
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[v][i] += sg * r1[u][i];
        }
      }
    }
  };
  // walk the list once: its length (up to CAP + 1), and entry t in slot t (written by lane
  // t mod G)
  int n_pos = 0;
  for (int e = static_cast<int>(q); e >= 0; e = next[e]) {
    if (n_pos < CAP && n_pos % G == l) s_list[grp][n_pos] = e;
    if (++n_pos > CAP) break;
  }
  if (n_pos == 1) {
    add(q);
  } else if (n_pos <= CAP) {
    // the group's lanes are one wave's: order the LDS writes before the other lanes' reads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int i = l; i < n_pos; i += G) {
      const int v = s_list[grp][i];
      int rank = 0;  // entries smaller than v (positions are distinct)
      for (int j = 0; j < n_pos; ++j) rank += s_list[grp][j] < v ? 1 : 0;
      s_sorted[grp][rank] = v;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int t = 0; t < n_pos; ++t) add(s_sorted[grp][t]);
  } else {
    // ascending scan of dst[]: lane l tests positions base + l·K + [0, K); the group's lanes
    // with hits are taken in lane order (ballot), each lane's hits in k order (its mask,
    // broadcast) — i.e. ascending positions, the order of the other paths
    constexpr int K = 16;
    const int P = static_cast<int>(3 * a.B);
    const int g0 = static_cast<int>(threadIdx.x & 63) - l;  // the group's first lane in the wave
    for (int base = 0; base < P; base += K * G) {
      unsigned hits = 0;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int e = base + l * K + k;
        if (e < P && dst[e] == r) hits |= 1u << k;
      }
      unsigned long long lanes = __ballot(hits != 0u);
      if (G < 64) lanes = (lanes >> g0) & ((1ull << G) - 1ull);
      while (lanes) {
        const int src = __ffsll(static_cast<unsigned long long>(lanes)) - 1;
        lanes &= lanes - 1ull;
        unsigned m = static_cast<unsigned>(__shfl(static_cast<int>(hits), g0 + src));
        while (m) {  // up to four positions at a time: their loads in flight together
          int64_t js[4];
          int cnt = 0;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            js[u] = 0;
            if (m) {
              js[u] = base + src * K + (__ffs(m) - 1);
              m &= m - 1u;
              ++cnt;
            }
          }
          add4(js, cnt);
        }
      }
    }
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c = 4 * (l + v * G);
    if (c >= a.d) break;
    store_vec<4>(dE + static_cast<int64_t>(r) * ldd + c, acc[v]);
  }
}

bool al16(const void* p, int64_t ld) {
  return reinterpret_cast<uintptr_t>(p) % 16 == 0 && ld % 4 == 0;
}

int group_for(int d) {
  const int lanes = d / 4;
  return lanes >= 64 ? 64 : (lanes >= 16 ? 16 : (lanes >= 4 ? 4 : 1));
}

hgd_status check(const BprArgs& a, const char* fn) {
  HGD_REQUIRE(a.B >= 1 && a.nu >= 1 && a.ni >= 1, "%s: empty batch or table", fn);
  HGD_REQUIRE(a.d >= 4 && a.d % 4 == 0 && a.d <= 256, "%s: d = %d (needs a multiple of 4 <= 256)",
              fn, a.d);
  HGD_REQUIRE(a.E && a.uid && a.pid && a.nid, "%s: null pointer", fn);
  HGD_REQUIRE(a.lde >= a.d && al16(a.E, a.lde), "%s: table rows must be 16-byte aligned", fn);
  HGD_REQUIRE(3 * a.B < 0x7fffffffLL && a.nu + a.ni < 0x7fffffffLL, "%s: too large", fn);
  return HGD_OK;
}

}  // namespace
}  // namespace hgd

using namespace hgd;

extern "C" size_t hgd_bpr_workspace_size(int64_t batch, int64_t n_rows) {
  const size_t b = static_cast<size_t>(batch > 0 ? batch : 0);
  return align_up(b * 4) + align_up(static_cast<size_t>(n_rows > 0 ? n_rows : 0) * 4) +
         2 * align_up(3 * b * 4);
}

extern "C" hgd_status hgd_bpr_forward(const float* E, int64_t lde, int64_t n_users,
                                      int64_t n_items, int32_t d, const int64_t* uid,
                                      const int64_t* pid, const int64_t* nid, int64_t batch,
                                      float* anc_out, float* pos_out, float* coef, float* loss,
                                      int32_t* bad_index, void* workspace,
                                      size_t workspace_bytes, void* stream) {
  clear_error();
  BprArgs a{E, lde, n_users, n_items, uid, pid, nid, batch, d};
  const hgd_status c = check(a, "hgd_bpr_forward");
  if (c != HGD_OK) return c;
  HGD_REQUIRE(coef && loss, "hgd_bpr_forward: null coef / loss");
  HGD_REQUIRE((!anc_out || reinterpret_cast<uintptr_t>(anc_out) % 16 == 0) &&
                  (!pos_out || reinterpret_cast<uintptr_t>(pos_out) % 16 == 0),
              "hgd_bpr_forward: outputs must be 16-byte aligned");
  const size_t need = hgd_bpr_workspace_size(batch, n_users + n_items);
  if (!workspace || workspace_bytes < need)
    return fail(HGD_ERR_WORKSPACE, "hgd_bpr_forward: workspace %zu < required %zu",
                workspace_bytes, need);
  float* term = static_cast<float*>(workspace);
  hipStream_t st = as_stream(stream);
  const int G = group_for(d);
  const unsigned blocks = static_cast<unsigned>((batch + kBlock / G - 1) / (kBlock / G));
  switch (G) {
    case 64: hipLaunchKernelGGL(k_bpr_rows<64>, dim3(blocks), dim3(kBlock), 0, st, a, anc_out, pos_out, term, coef, bad_index); break;
    case 16: hipLaunchKernelGGL(k_bpr_rows<16>, dim3(blocks), dim3(kBlock), 0, st, a, anc_out, pos_out, term, coef, bad_index); break;
    case 4: hipLaunchKernelGGL(k_bpr_rows<4>, dim3(blocks), dim3(kBlock), 0, st, a, anc_out, pos_out, term, coef, bad_index); break;
    default: hipLaunchKernelGGL(k_bpr_rows<1>, dim3(blocks), dim3(kBlock), 0, st, a, anc_out, pos_out, term, coef, bad_index); break;
  }
  hgd_status s = check_launch("hgd_bpr_forward rows");
  if (s != HGD_OK) return s;
  hipLaunchKernelGGL(k_bpr_mean, dim3(1), dim3(1024), 0, st, term, batch, loss);
  return check_launch("hgd_bpr_forward mean");
}

extern "C" hgd_status hgd_bpr_backward(const float* E, int64_t lde, int64_t n_users,
                                       int64_t n_items, int32_t d, const int64_t* uid,
                                       const int64_t* pid, const int64_t* nid, int64_t batch,
                                       const float* coef, const float* grad, float* dE,
                                       int64_t ldd, void* workspace, size_t workspace_bytes,
                                       void* stream) {
  clear_error();
  BprArgs a{E, lde, n_users, n_items, uid, pid, nid, batch, d};
  const hgd_status c = check(a, "hgd_bpr_backward");
  if (c != HGD_OK) return c;
  HGD_REQUIRE(coef && grad && dE, "hgd_bpr_backward: null coef / grad / dE");
  HGD_REQUIRE(ldd >= d && al16(dE, ldd), "hgd_bpr_backward: dE rows must be 16-byte aligned");
  const size_t need = hgd_bpr_workspace_size(batch, n_users + n_items);
  if (!workspace || workspace_bytes < need)
    return fail(HGD_ERR_WORKSPACE, "hgd_bpr_backward: workspace %zu < required %zu",
                workspace_bytes, need);
  const int64_t N = n_users + n_items;
  char* w = static_cast<char*>(workspace) + align_up(static_cast<size_t>(batch) * 4);
  int* head = reinterpret_cast<int*>(w);
  w += align_up(static_cast<size_t>(N) * 4);
  int* next = reinterpret_cast<int*>(w);
  int* dst = reinterpret_cast<int*>(w + align_up(static_cast<size_t>(3 * batch) * 4));
  hipStream_t st = as_stream(stream);
  const int64_t init_n = std::max<int64_t>(N * (d / 4), N);
  hipLaunchKernelGGL(k_bpr_bwd_init, dim3(grid_for(init_n)), dim3(kBlock), 0, st, dE, ldd, N, d,
                     head);
  hipLaunchKernelGGL(k_bpr_bwd_link, dim3(grid_for(3 * batch)), dim3(kBlock), 0, st, a, head,
                     next, dst);
  const int G = group_for(d);
  const unsigned blocks = static_cast<unsigned>((3 * batch + kBlock / G - 1) / (kBlock / G));
  switch (G) {
    case 64: hipLaunchKernelGGL(k_bpr_bwd_rows<64>, dim3(blocks), dim3(kBlock), 0, st, a, coef, grad, head, next, dst, dE, ldd); break;
    case 16: hipLaunchKernelGGL(k_bpr_bwd_rows<16>, dim3(blocks), dim3(kBlock), 0, st, a, coef, grad, head, next, dst, dE, ldd); break;
    case 4: hipLaunchKernelGGL(k_bpr_bwd_rows<4>, dim3(blocks), dim3(kBlock), 0, st, a, coef, grad, head, next, dst, dE, ldd); break;
    default: hipLaunchKernelGGL(k_bpr_bwd_rows<1>, dim3(blocks), dim3(kBlock), 0, st, a, coef, grad, head, next, dst, dE, ldd); break;
  }
  return check_launch("hgd_bpr_backward");
}
