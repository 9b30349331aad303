// BPR loss of a recommender batch straight from the embedding table (util/loss_torch.py:5-9 on
// the rows model/graph/HCCF.py:84-86 gathers):
//   anc = E[uid], pos = E[nu + pid], neg = E[nu + nid]
//   loss = mean_k −log(1e-5 + σ(⟨anc_k, pos_k⟩ − ⟨anc_k, neg_k⟩))
// In the reference these are three index gathers, two mul + sum pairs, sub, sigmoid, add, log,
// neg and mean forward, and the same chain backward ending in three sort-based index_put
// scatters (~40 small launches per step). Here: forward = one row kernel (gather, both dots,
// per-row term and backward coefficient) + one fixed-order reduction; backward = zero/init,
// one pass linking every position into its destination row's list and counting the row
// (integer atomics), one row kernel in which one position per destination sums the
// contributions of a row's (at most kWalkMax) positions in ascending position order, and one
// kernel for the rows with more positions (one workgroup per row, fixed contiguous ranges of
// its ascending positions, partials combined in range order) — deterministic, no float
// atomics, no sort.
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

constexpr int kWalkMax = 8;          // rows with at most this many positions walk their list
constexpr int kHeavyGrid = 256;       // blocks of the heavy-row kernel (they loop over the rows)
constexpr int kWin = 16 * kBlock;     // positions one heavy-row window scans (16 per thread)

__device__ __forceinline__ int64_t batch_row(const BprArgs& a, int64_t j) {
  return j < a.B ? j : (j < 2 * a.B ? j - a.B : j - 2 * a.B);
}

__global__ void k_bpr_bwd_init(float* dE, int64_t lde, int64_t n_rows, int32_t d, int* head,
                               int* cnt, int* n_heavy) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t per = d / 4;
  if (i < n_rows * per) {
    const int64_t r = i / per, c = 4 * (i % per);
    const float z[4] = {0.f, 0.f, 0.f, 0.f};
    store_vec<4>(dE + r * lde + c, z);
  }
  if (i < n_rows) {
    head[i] = -1;
    cnt[i] = 0;
  }
  if (i == 0) *n_heavy = 0;
}

// Every position pushes itself onto its destination row's list (integer atomics; the list
// ORDER depends on timing, the set does not — the row kernel sorts it) and counts itself; the
// position that takes a row past kWalkMax enters the row in the heavy list (exactly once).
__global__ void k_bpr_bwd_link(BprArgs a, int* head, int* next, int* dst, int* cnt, int* heavy,
                               int* n_heavy) {
  const int64_t q = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (q >= 3 * a.B) return;
  const int r = static_cast<int>(dest_row(a, q));
  dst[q] = r;
  next[q] = atomicExch(head + r, static_cast<int>(q));
  if (atomicAdd(cnt + r, 1) == kWalkMax) heavy[atomicAdd(n_heavy, 1)] = r;
}

// One lane group per position; the position left at the head of each destination row's list
// writes that row when the row has at most kWalkMax positions (the heavy kernel writes the
// others): the contributions of all its positions, summed in ascending position order — the
// list walked once into the group's LDS slots, ranked there (each lane counts the smaller
// entries of its slots), added in rank order.
template <int G>
__global__ __launch_bounds__(kBlock) void k_bpr_bwd_rows(BprArgs a, const float* coef,
                                                        const float* grad, const int* head,
                                                        const int* next, const int* dst,
                                                        const int* cnt, float* dE, int64_t ldd) {
  constexpr int GPB = kBlock / G;
  const int l = threadIdx.x % G;
  const int64_t q = static_cast<int64_t>(blockIdx.x) * GPB + threadIdx.x / G;
  if (q >= 3 * a.B) return;
  __shared__ int s_list[GPB][kWalkMax];
  __shared__ int s_sorted[GPB][kWalkMax];
  const int grp = threadIdx.x / G;
  const int r = dst[q];
  if (head[r] != static_cast<int>(q)) return;  // group-uniform
  const int n_pos = cnt[r];
  if (n_pos > kWalkMax) return;  // the heavy kernel's row
  const float gB = -(*grad) / static_cast<float>(a.B);
  constexpr int NV = 4;  // float4 column blocks per lane: d / 4 <= NV·G for every group_for(d)
  float acc[NV][4];
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[v][i] = 0.f;
  auto add = [&](int64_t j) {
    const int64_t k = batch_row(a, j);
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
  if (n_pos == 1) {
    add(q);
  } else {
    int e = static_cast<int>(q);
    for (int t = 0; t < n_pos; ++t, e = next[e])
      if (t % G == l) s_list[grp][t] = e;
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
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c = 4 * (l + v * G);
    if (c >= a.d) break;
    store_vec<4>(dE + static_cast<int64_t>(r) * ldd + c, acc[v]);
  }
}

// The rows with more than kWalkMax positions (a skewed catalogue's popular items: under
// Zipf(1.2) popularity one item is the positive of ~740 of 4,096 rows), one workgroup per row
// (the blocks loop over the heavy list). Per window of kWin positions (of the anchors for a user
// row, of the positives and negatives for an item row): every thread tests its
// 16 consecutive positions against the row, a block scan of the hit counts writes the row's
// positions to LDS in ascending order, the GPB lane groups sum contiguous ranges of them (U rows
// loaded before they are added) and group 0 adds the group partials in group order to the row.
// The order is fixed by (batch, d), so the result is deterministic; every load of a window is
// independent, where one lane group walking the row's list — or scanning the batch alone — paid
// a dependent load per position (the round-4 scan path took ~0.5 ms on that batch).
template <int G>
__global__ __launch_bounds__(kBlock) void k_bpr_bwd_heavy(BprArgs a, const float* coef,
                                                         const float* grad, const int* dst,
                                                         const int* heavy, const int* n_heavy,
                                                         float* dE, int64_t ldd) {
  constexpr int GPB = kBlock / G;
  constexpr int NV = 4;
  constexpr int U = 8;
  __shared__ int s_hits[kWin];
  __shared__ int s_wave[kBlock / 64];
  __shared__ float s_part[GPB][NV * G * 4];
  const int tid = threadIdx.x, l = tid % G, grp = tid / G;
  const int lane = tid & 63, wave = tid >> 6;
  const float gB = -(*grad) / static_cast<float>(a.B);
  const int P = static_cast<int>(3 * a.B);
  const int nh = *n_heavy;
  for (int h = blockIdx.x; h < nh; h += gridDim.x) {
    const int r = heavy[h];
    float acc[NV][4];
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[v][i] = 0.f;
    // a user row is only ever an anchor's destination, an item row a positive's or a
    // negative's: scan that part of the batch
    const int p_lo = r < a.nu ? 0 : static_cast<int>(a.B);
    const int p_hi = r < a.nu ? static_cast<int>(a.B) : P;
    for (int base = p_lo; base < p_hi; base += kWin) {
      const int p0 = base + 16 * tid;
      unsigned m = 0;
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (p0 + k < p_hi && dst[p0 + k] == r) m |= 1u << k;
      const int c = __popc(m);
      int incl = c;  // inclusive scan over the wave, then the waves in order
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
      }
      if (lane == 63) s_wave[wave] = incl;
      __syncthreads();
      int off = 0, n = 0;
#pragma unroll
      for (int w = 0; w < kBlock / 64; ++w) {
        const int t = s_wave[w];
        off += w < wave ? t : 0;
        n += t;
      }
      int pos = off + incl - c;
      while (m) {
        s_hits[pos++] = p0 + __ffs(m) - 1;
        m &= m - 1u;
      }
      __syncthreads();
      if (n == 0) continue;  // block-uniform
      const int lo = static_cast<int>(static_cast<int64_t>(n) * grp / GPB);
      const int hi = static_cast<int>(static_cast<int64_t>(n) * (grp + 1) / GPB);
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int cc = 4 * (l + v * G);
        if (cc >= a.d) break;
        float part[4] = {0.f, 0.f, 0.f, 0.f};
        for (int t0 = lo; t0 < hi; t0 += U) {
          float r1[U][4], r2[U][4], tt[U];
          bool anc[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            anc[u] = false;
            tt[u] = 0.f;
            if (t0 + u < hi) {
              const int64_t j = s_hits[t0 + u];
              const int64_t k = batch_row(a, j);
              const float t = gB * coef[k];
              anc[u] = j < a.B;
              if (anc[u]) {
                tt[u] = t;
                load_vec<4>(a.E + static_cast<int64_t>(dst[a.B + k]) * a.lde + cc, r1[u]);
                load_vec<4>(a.E + static_cast<int64_t>(dst[2 * a.B + k]) * a.lde + cc, r2[u]);
              } else {
                tt[u] = j < 2 * a.B ? t : -t;
                load_vec<4>(a.E + static_cast<int64_t>(dst[k]) * a.lde + cc, r1[u]);
              }
            }
          }
#pragma unroll
          for (int u = 0; u < U; ++u) {
            if (t0 + u < hi) {
              if (anc[u]) {
#pragma unroll
                for (int i = 0; i < 4; ++i) part[i] += tt[u] * (r1[u][i] - r2[u][i]);
              } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) part[i] += tt[u] * r1[u][i];
              }
            }
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) s_part[grp][4 * (l + v * G) + i] = part[i];
      }
      __syncthreads();
      if (grp == 0) {
        for (int s = 0; s < GPB; ++s) {
#pragma unroll
          for (int v = 0; v < NV; ++v) {
            const int cc = 4 * (l + v * G);
            if (cc >= a.d) break;
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[v][i] += s_part[s][cc + i];
          }
        }
      }
      __syncthreads();  // s_hits / s_part are refilled by the next window
    }
    if (grp == 0) {
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int cc = 4 * (l + v * G);
        if (cc >= a.d) break;
        store_vec<4>(dE + static_cast<int64_t>(r) * ldd + cc, acc[v]);
      }
    }
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
  const size_t n = static_cast<size_t>(n_rows > 0 ? n_rows : 0);
  // term | head | next | dst | cnt | n_heavy | heavy rows
  return align_up(b * 4) + align_up(n * 4) + 2 * align_up(3 * b * 4) + align_up(n * 4) +
         align_up(4) + align_up((3 * b / (kWalkMax + 1) + 1) * 4);
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
  w += align_up(static_cast<size_t>(3 * batch) * 4);
  int* dst = reinterpret_cast<int*>(w);
  w += align_up(static_cast<size_t>(3 * batch) * 4);
  int* cnt = reinterpret_cast<int*>(w);
  w += align_up(static_cast<size_t>(N) * 4);
  int* n_heavy = reinterpret_cast<int*>(w);
  int* heavy = reinterpret_cast<int*>(w + align_up(4));
  hipStream_t st = as_stream(stream);
  const int64_t init_n = std::max<int64_t>(N * (d / 4), N);
  hipLaunchKernelGGL(k_bpr_bwd_init, dim3(grid_for(init_n)), dim3(kBlock), 0, st, dE, ldd, N, d,
                     head, cnt, n_heavy);
  hipLaunchKernelGGL(k_bpr_bwd_link, dim3(grid_for(3 * batch)), dim3(kBlock), 0, st, a, head,
                     next, dst, cnt, heavy, n_heavy);
  const int G = group_for(d);
  const unsigned blocks = static_cast<unsigned>((3 * batch + kBlock / G - 1) / (kBlock / G));
#define HGD_BPR_ROWS(GG)                                                                        \
  hipLaunchKernelGGL(k_bpr_bwd_rows<GG>, dim3(blocks), dim3(kBlock), 0, st, a, coef, grad, head, \
                     next, dst, cnt, dE, ldd);                                                   \
  hipLaunchKernelGGL(k_bpr_bwd_heavy<GG>, dim3(kHeavyGrid), dim3(kBlock), 0, st, a, coef, grad, \
                     dst, heavy, n_heavy, dE, ldd)
  switch (G) {
    case 64: HGD_BPR_ROWS(64); break;
    case 16: HGD_BPR_ROWS(16); break;
    case 4: HGD_BPR_ROWS(4); break;
    default: HGD_BPR_ROWS(1); break;
  }
#undef HGD_BPR_ROWS
  return check_launch("hgd_bpr_backward");
}
